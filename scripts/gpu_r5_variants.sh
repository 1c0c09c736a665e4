#!/bin/bash
# Round 5: interleaved A/B of prebuilt .so variants (variants/_C_v*.so, built here with
# TFD_HIP_FLAGS=-D...): each is copied over the in-tree extension, checked by the fp32 numerics
# tests, then timed by the driver-style bench (VAR_BENCH overrides the bench arguments).
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
VARS=${VARS:-"0 1 2 3"}
ARGS=${VAR_BENCH:-"--dtype fp32 --steps 1000 --warmup 100"}
for v in $VARS; do
  cp variants/_C_v$v.so tensorflow_distributed_amd/_C.so || exit 1
  timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${VAR_TESTS:-tests/test_mnist_fp32_gpu.py} > gpurun_out/var_t$v.log 2>&1 || { echo "v$v tests failed"; tail -20 gpurun_out/var_t$v.log; exit 1; }
done
for r in 1 2 3; do
  for v in $VARS; do
    cp variants/_C_v$v.so tensorflow_distributed_amd/_C.so || exit 1
    timeout -k 10 120 python bench.py $ARGS > gpurun_out/var_b$v.log 2>&1 || { echo "v$v bench failed"; tail -5 gpurun_out/var_b$v.log; exit 1; }
    echo "run $r v$v: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/var_b$v.log)"
  done
done
