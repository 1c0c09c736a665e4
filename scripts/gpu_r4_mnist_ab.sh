#!/bin/bash
# MNIST A/B: the in-tree build (new) against build_ab/old (the previous commit's build), interleaved,
# after the MNIST engine GPU tests of the new build.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_mnist_engine_gpu.py} -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_mab_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r4_mab_tests.log | head -20; tail -30 gpurun_out/r4_mab_tests.log; exit 1; }
tail -1 gpurun_out/r4_mab_tests.log
ROOT=$(pwd)
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps ${STEPS:-1000} --warmup 200 > gpurun_out/r4_mab_new$i.log 2>&1 || { tail -20 gpurun_out/r4_mab_new$i.log; exit 1; }
  (cd build_ab/old && timeout -k 10 120 python bench.py --steps ${STEPS:-1000} --warmup 200) > gpurun_out/r4_mab_old$i.log 2>&1 || { tail -20 gpurun_out/r4_mab_old$i.log; exit 1; }
  echo "run $i new $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4_mab_new$i.log) old $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4_mab_old$i.log)"
done
if [ -n "$PROF" ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mab -o run -- python bench.py --steps 300 --warmup 100 > gpurun_out/r4_mab_prof.log 2>&1 || { tail -20 gpurun_out/r4_mab_prof.log; exit 1; }
  echo profiled
fi
