#!/bin/bash
# GPU test suite (optionally a subset: TESTS="tests/x.py -k y"), then optional bench lines.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-t}
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed: $?"; grep -E "PASS|FAIL|ERROR|Error|error" gpurun_out/pytest_gpu_$TAG.log | tail -40; tail -60 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_gpu_$TAG.log | tail -80
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; cat gpurun_out/bench_$TAG.log; exit 1; }
  cat gpurun_out/bench_$TAG.log | grep -v amdgpu.ids
  timeout -k 10 120 python bench.py --steps 1000 --warmup 100 > gpurun_out/bench_long_$TAG.log 2>&1 || { echo "bench failed"; cat gpurun_out/bench_long_$TAG.log; exit 1; }
  cat gpurun_out/bench_long_$TAG.log | grep -v amdgpu.ids
fi
