#!/bin/bash
# Round 5: kernel table + per-step timeline of the fp32 (reference-precision) MNIST step.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 120 python bench.py --dtype fp32 --steps 1000 --warmup 100 > gpurun_out/r5_f32_b.log 2>&1 || { tail gpurun_out/r5_f32_b.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_f32_b.log
rm -rf gpurun_out/r5_prof_f32
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_prof_f32 -o run -- python3 bench.py --dtype fp32 --steps 300 --warmup 20 --phases 0 --min_warmup_ms 0 --state_steps 0 > gpurun_out/r5_prof_f32.log 2>&1 || { tail gpurun_out/r5_prof_f32.log; exit 1; }
db=$(find gpurun_out/r5_prof_f32 -name "*.db" | head -1)
python scripts/prof_summary.py $db --min-calls 100
python scripts/prof_timeline.py $db --anchor mnist_adam | tail -12
