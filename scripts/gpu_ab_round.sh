#!/bin/bash
# GPU tests for the MNIST engine / ResNet, MNIST A/B (fc-region bf16 grads on one GPU), ResNet-50
# b128 bench. Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-ab}
timeout -k 10 400 python -u -m pytest tests/test_mnist_engine_gpu.py tests/test_resnet_gpu.py tests/test_conv_ops_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
for v in 0 1 0 1; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --local_bf16_grads $v > gpurun_out/bench_${TAG}_bf$v.log 2>&1 \
    || { echo "bench failed"; cat gpurun_out/bench_${TAG}_bf$v.log; exit 1; }
  echo "local_bf16_grads=$v: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_${TAG}_bf$v.log)"
done
timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 10 --warmup 3 > gpurun_out/bench_r50_$TAG.log 2>&1 \
  || { echo "bench r50 failed"; tail -30 gpurun_out/bench_r50_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_r50_$TAG.log
