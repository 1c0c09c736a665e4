#!/bin/bash
# Conflict-free LDS images in the generic GEMM core (gemm.h swz_chunk / pad 16): tests, MNIST A/B vs
# TFD_LDS_SWZ=0, ResNet-50 A/B (swz, no-swz, and --bn_final_side 0).
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mnist_engine_gpu.py tests/test_conv_ops_gpu.py tests/test_resnet_gpu.py tests/test_dropout_curve_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_swz.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/pytest_swz.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/pytest_swz.log)"
ROUNDS=3 TAG=swz ARMS="base|base|;noswz|noswz|" bash scripts/gpu_ab3.sh || exit 1
lib() { if [ "$1" = "base" ]; then echo $PWD/tensorflow_distributed_amd/_C.so; else echo $PWD/tensorflow_distributed_amd/_C_$1.so; fi; }
for r in 1 2; do
  for arm in "base|" "noswz|" "base|--bn_final_side 0"; do
    IFS='|' read -r l args <<< "$arm"
    TFD_NATIVE_LIB=$(lib $l) timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 $args > gpurun_out/rnswz.tmp 2>&1 \
      || { echo "resnet bench failed"; tail -20 gpurun_out/rnswz.tmp; exit 1; }
    echo "rn50 $l $args $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rnswz.tmp)" | tee -a gpurun_out/ab_rnswz.log
  done
done
