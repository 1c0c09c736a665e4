#!/bin/bash
# Quick GPU iteration: numerics tests + 1-GPU bench + rocprofv3 kernel stats summary.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-cur}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; cat gpurun_out/bench_$TAG.log; exit 1; }
cat gpurun_out/bench_$TAG.log
rm -rf gpurun_out/prof_$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 200 --warmup 20 ${BENCH_ARGS:-} > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof_$TAG.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof_$TAG -name "*.db" | head -1) | tee gpurun_out/kernels_$TAG.txt
