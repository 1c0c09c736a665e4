#!/bin/bash
# Forward BN fold: conv-op + ResNet numerics, then ResNet-50 b128 with the fold off / on and a kernel
# trace of the folded step.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv_ops_gpu.py tests/test_resnet_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_fold_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r4_fold_tests.log | head -20; tail -30 gpurun_out/r4_fold_tests.log; exit 1; }
tail -1 gpurun_out/r4_fold_tests.log
for f in 0 1 2; do
  timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 --fold_bn $f > gpurun_out/r4_rn50_fold$f.log 2>&1 || { tail -20 gpurun_out/r4_rn50_fold$f.log; exit 1; }
  echo "fold_bn=$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4_rn50_fold$f.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fold -o run -- python bench_resnet.py --depth 50 --batch_size 128 --steps 15 --warmup 3 --fold_bn ${PROF_FOLD:-1} > gpurun_out/r4_fold_prof.log 2>&1 || { tail -20 gpurun_out/r4_fold_prof.log; exit 1; }
echo profiled
