#!/bin/bash
# Round 5: weight-gradient split-count A/B (variants/_C_v*.so built with -DTFD_WG_MINPX / -DTFD_WG_BLOCKS):
# wgrad numerics per variant, then 3 interleaved rounds of ResNet-50 b128 and ResNet-18 steps.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
VARS=${VARS:-"0 1 2 3 4"}
for v in $VARS; do
  cp variants/_C_v$v.so tensorflow_distributed_amd/_C.so || exit 1
  timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_ops_gpu.py -k "${TESTK:-wgrad}" > gpurun_out/ws_t$v.log 2>&1 || { echo "v$v tests failed"; tail -20 gpurun_out/ws_t$v.log; exit 1; }
done
for r in 1 2 3; do
  for v in $VARS; do
    cp variants/_C_v$v.so tensorflow_distributed_amd/_C.so || exit 1
    timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/ws_b$v.log 2>&1 || { echo "v$v bench failed"; tail -5 gpurun_out/ws_b$v.log; exit 1; }
    timeout -k 10 300 python bench_resnet.py --depth 18 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/ws_c$v.log 2>&1 || { echo "v$v r18 bench failed"; tail -5 gpurun_out/ws_c$v.log; exit 1; }
    echo "run $r v$v: r50 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ws_b$v.log) r18 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ws_c$v.log)"
  done
done
