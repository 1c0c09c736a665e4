#!/bin/bash
# Round 5: split-K heuristics of the 256-row core's weight gradients (variants/_C_v*.so built with
# -DTFD_G256_WG_MINPX / -DTFD_G256_WG_TARGET): wgrad numerics on that core, then the per-layer probe.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in ${VARS:-0 1 2 3 4}; do
  cp variants/_C_v$v.so tensorflow_distributed_amd/_C.so || exit 1
  timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_ops_gpu.py -k "wgrad" > gpurun_out/gw_t$v.log 2>&1 || { echo "v$v tests failed"; tail -20 gpurun_out/gw_t$v.log; exit 1; }
  echo "v$v tests: $(tail -1 gpurun_out/gw_t$v.log)"
  timeout -k 10 200 python scripts/debug/gemm_probe.py --only wgrad --torch 0 > gpurun_out/gw_p$v.log 2>&1 || { echo "v$v probe failed"; tail -20 gpurun_out/gw_p$v.log; exit 1; }
  grep -v "dense4096\|amdgpu.ids" gpurun_out/gw_p$v.log | sed "s/^/v$v /" | sed 's/| torch.*//'
done
