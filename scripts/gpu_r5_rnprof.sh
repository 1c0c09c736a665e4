#!/bin/bash
# Round 5: ResNet-50 B=128 kernel table at HEAD (rocprofv3 --kernel-trace --stats).
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -rf gpurun_out/r5_prof_rn
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_prof_rn -o run -- python3 bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/r5_prof_rn.log 2>&1 || { tail -20 gpurun_out/r5_prof_rn.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_prof_rn.log
db=$(find gpurun_out/r5_prof_rn -name "*.db" | head -1)
python scripts/prof_summary.py $db --min-calls 20 > gpurun_out/r5_rn_kernels.txt
head -45 gpurun_out/r5_rn_kernels.txt
rm -rf gpurun_out/r5_prof_rn
