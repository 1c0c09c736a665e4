#!/bin/bash
# One GPU-box session: GPU test suite, 1-GPU headline bench, rocprofv3 kernel stats, and the
# same-hardware PyTorch reference path (scripts/bench_torch_ref.py). Every GPU step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed: $?"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 > gpurun_out/bench_$TAG.log 2>&1 \
  || { echo "bench failed"; cat gpurun_out/bench_$TAG.log; exit 1; }
cat gpurun_out/bench_$TAG.log
rm -rf gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 200 --warmup 20 \
  > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof_$TAG.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof_$TAG -name "*.db" | head -1) --min-calls 100 > gpurun_out/kernels_$TAG.txt || true
cat gpurun_out/kernels_$TAG.txt
if [ "${TORCHREF:-1}" = "1" ]; then
  timeout -k 10 300 python scripts/bench_torch_ref.py --model mnist --batch_size 128 --steps 500 \
    > gpurun_out/torchref_mnist_$TAG.log 2>&1 || { echo "torch ref failed"; tail -20 gpurun_out/torchref_mnist_$TAG.log; exit 1; }
  cat gpurun_out/torchref_mnist_$TAG.log
  timeout -k 10 300 python scripts/bench_torch_ref.py --model resnet50 --batch_size 64 --steps 10 --warmup 3 \
    > gpurun_out/torchref_r50_$TAG.log 2>&1 || { echo "torch ref r50 failed"; tail -20 gpurun_out/torchref_r50_$TAG.log; exit 1; }
  cat gpurun_out/torchref_r50_$TAG.log
fi
