#!/bin/bash
# Round 5: ResNet weight-gradient GEMM variants (variants/_C_v*.so built with TFD_HIP_FLAGS=-DTFD_WG_*):
# numerics, per-layer wgrad probe, then interleaved ResNet-50 b128 steps.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
VARS=${VARS:-"0 1 2 3 4 5"}
for v in $VARS; do
  cp variants/_C_v$v.so tensorflow_distributed_amd/_C.so || exit 1
  timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_ops_gpu.py -k "wgrad" > gpurun_out/wg_t$v.log 2>&1 || { echo "v$v tests failed"; tail -20 gpurun_out/wg_t$v.log; exit 1; }
  echo "v$v tests: $(tail -1 gpurun_out/wg_t$v.log)"
  timeout -k 10 200 python scripts/debug/gemm_probe.py --only wgrad --torch 0 > gpurun_out/wg_p$v.log 2>&1 || { echo "v$v probe failed"; tail -20 gpurun_out/wg_p$v.log; exit 1; }
  grep -v dense4096 gpurun_out/wg_p$v.log | sed "s/^/v$v /"
done
for r in 1 2; do
  for v in $VARS; do
    cp variants/_C_v$v.so tensorflow_distributed_amd/_C.so || exit 1
    timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/wg_b$v.log 2>&1 || { echo "v$v bench failed"; tail -5 gpurun_out/wg_b$v.log; exit 1; }
    echo "run $r v$v: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/wg_b$v.log)"
  done
done
