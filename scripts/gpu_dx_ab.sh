#!/bin/bash
# fc1 dX tile width A/B: engine tests, then fused one-GPU and forced-DP (8-GPU default) step times, 3 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/tensorflow_distributed_amd
for lib in _C _C_dx32; do
  TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 300 python -u -m pytest tests/test_mnist_engine_gpu.py tests/test_dp_transport_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "not bench and not quickstart and not dist_main" > gpurun_out/pt_dx_$lib.log 2>&1 || { echo "pytest $lib failed"; tail -30 gpurun_out/pt_dx_$lib.log; exit 1; }
  echo "tests $lib: $(tail -1 gpurun_out/pt_dx_$lib.log)"
done
for r in 1 2 3; do
  for lib in _C _C_dx32; do
    TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --phases 0 > gpurun_out/dx.log 2>&1 || { echo "bench failed"; tail gpurun_out/dx.log; exit 1; }
    one=$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dx.log)
    TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --phases 0 --force_dp 1 --zero 1 > gpurun_out/dx.log 2>&1 || { echo "bench dp failed"; tail gpurun_out/dx.log; exit 1; }
    echo "$r $lib one-GPU $one | forced-DP $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dx.log)"
  done
done
