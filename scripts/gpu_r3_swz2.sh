#!/bin/bash
# A/Bs first (MNIST swz, ResNet swz / side finalize), then the RCCL ResNet probe with and without the side finalize.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
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
timeout -k 10 300 python -u -m pytest tests/test_mnist_engine_gpu.py tests/test_conv_ops_gpu.py tests/test_dropout_curve_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_swz.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/pytest_swz.log; exit 1; }
echo "mnist/conv tests: $(tail -1 gpurun_out/pytest_swz.log)"
timeout -k 10 90 python scripts/debug/rccl_resnet_probe.py 0 0 > gpurun_out/probe_noside.log 2>&1; echo "probe no side rc=$?"; tail -3 gpurun_out/probe_noside.log
timeout -k 10 90 python scripts/debug/rccl_resnet_probe.py 0 1 > gpurun_out/probe_side.log 2>&1; echo "probe side rc=$?"; tail -30 gpurun_out/probe_side.log
