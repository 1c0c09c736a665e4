#!/bin/bash
# One GPU-box session: numerics tests, 1-GPU bench (graph + eager), rocprofv3 kernel stats.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
STEPS=${STEPS:-500}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed: $?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps $STEPS > gpurun_out/bench_graph.log 2>&1 || { echo "bench failed"; cat gpurun_out/bench_graph.log; exit 1; }
cat gpurun_out/bench_graph.log
timeout -k 10 300 python bench.py --eager --steps 200 > gpurun_out/bench_eager.log 2>&1 || { echo "eager bench failed"; cat gpurun_out/bench_eager.log; exit 1; }
cat gpurun_out/bench_eager.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 200 --warmup 20 > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name "*stats*" | head
