#!/bin/bash
# Round-3 check at HEAD: full GPU suite, value-state A/B (learnable step-100 vs collapsed random
# labels, zero-skip on/off), self-launched 2/4-rank benches, 1-GPU kernel table.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed: $?"; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
ROUNDS=2 TAG=state ARMS="base100|base|--data strokes --state_steps 100;skip100|skip0|--data strokes --state_steps 100;rnd0|base|--data random --state_steps 0;skiprnd0|skip0|--data random --state_steps 0" bash scripts/gpu_ab3.sh || exit 1
for n in 2 4; do
  timeout -k 10 240 python bench.py --gpus $n --steps 200 --warmup 20 > gpurun_out/bench_g$n.log 2>&1 || { echo "bench gpus $n failed"; tail -30 gpurun_out/bench_g$n.log; exit 1; }
  tail -2 gpurun_out/bench_g$n.log
done
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_drv.log 2>&1 && cat gpurun_out/bench_drv.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 200 --warmup 20 --phases 0 > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof -name "*.db" | head -1) > gpurun_out/kernels.txt 2>&1; cat gpurun_out/kernels.txt | head -30
rm -rf gpurun_out/prof
