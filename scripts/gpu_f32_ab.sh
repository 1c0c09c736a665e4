#!/bin/bash
# fp32 engine variants: fp32 numerics tests under each lib, then bench --dtype fp32 (1000/100), 2 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/tensorflow_distributed_amd
for lib in ${LIBS:-_C _C_fbk64}; do
  TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 300 python -u -m pytest tests/test_mnist_fp32_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_f32_$lib.log 2>&1 || { echo "pytest $lib failed"; tail -30 gpurun_out/pytest_f32_$lib.log; exit 1; }
  echo "tests $lib: $(tail -1 gpurun_out/pytest_f32_$lib.log)"
done
for r in 1 2; do
  for lib in ${LIBS:-_C _C_fbk64}; do
    TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 120 python bench.py --dtype fp32 --steps 1000 --warmup 100 --phases 0 > gpurun_out/f32ab.log 2>&1 || { echo "bench $lib failed"; tail gpurun_out/f32ab.log; exit 1; }
    echo "$r $lib: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/f32ab.log)"
  done
done
