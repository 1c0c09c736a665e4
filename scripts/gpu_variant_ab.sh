#!/bin/bash
# Interleaved A/B of native-library variants (tensorflow_distributed_amd/_C_<name>.so, "base" = _C.so):
# engine numerics tests under each variant first, then 3 rounds of 1-GPU bench per variant.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-vab}
lib() { if [ "$1" = "base" ]; then echo $PWD/tensorflow_distributed_amd/_C.so; else echo $PWD/tensorflow_distributed_amd/_C_$1.so; fi; }
for v in ${VARIANTS:-base}; do
  [ "${SKIP_TESTS:-0}" = "1" ] && break
  TFD_NATIVE_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest tests/test_mnist_engine_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_${TAG}_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 gpurun_out/pytest_${TAG}_$v.log; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/pytest_${TAG}_$v.log)"
done
for r in 1 2 3; do
  for v in ${VARIANTS:-base}; do
    TFD_NATIVE_LIB=$(lib $v) timeout -k 10 120 python bench.py --steps 2000 --warmup 200 > gpurun_out/ab_$TAG.tmp 2>&1 \
      || { echo "bench $v failed"; cat gpurun_out/ab_$TAG.tmp; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$TAG.tmp)" | tee -a gpurun_out/ab_$TAG.log
  done
done
