#!/bin/bash
# MNIST headline bench (A/B-free) + ResNet-50 b128 bench, each under its own time limit.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-mr}
timeout -k 10 300 python -u -m pytest tests/test_mnist_engine_gpu.py tests/test_runner_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 \
  || { echo "pytest failed"; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/bench_${TAG}_$i.log 2>&1 || { echo "bench failed"; cat gpurun_out/bench_${TAG}_$i.log; exit 1; }
  echo "mnist: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_${TAG}_$i.log)"
done
for i in 1 2; do
  timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 30 --warmup 5 > gpurun_out/bench_r50_${TAG}_$i.log 2>&1 || { echo "r50 failed"; tail -20 gpurun_out/bench_r50_${TAG}_$i.log; exit 1; }
  echo "r50: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_r50_${TAG}_$i.log)"
done
