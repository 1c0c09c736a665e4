#!/bin/bash
# ResNet library-variant A/B: conv/ResNet tests under each lib, then ResNet-50 and -18 ms/step, 2 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/tensorflow_distributed_amd
for lib in ${LIBS:-_C}; do
  TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 300 python -u -m pytest tests/test_conv_ops_gpu.py tests/test_resnet_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_rl_$lib.log 2>&1 || { echo "pytest $lib failed"; tail -30 gpurun_out/pytest_rl_$lib.log; exit 1; }
  echo "tests $lib: $(tail -1 gpurun_out/pytest_rl_$lib.log)"
done
for r in 1 2; do
  for lib in ${LIBS:-_C}; do
    for d in 50 18; do
      TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 300 python bench_resnet.py --depth $d --batch_size 128 --steps 10 --warmup 3 > gpurun_out/rl.log 2>&1 || { echo "bench $lib failed"; tail -20 gpurun_out/rl.log; exit 1; }
      echo "$r $lib r$d: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rl.log | head -1)"
    done
  done
done
