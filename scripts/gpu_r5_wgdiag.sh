#!/bin/bash
# Round 5: timing-diagnosis builds of the weight-gradient GEMM (variants/_C_v*.so: v0 HEAD, then with
# the K-loop's global loads / MFMA sweep / atomic epilogue removed) on the per-layer wgrad probe.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in ${VARS:-0 1 2 3 4}; do
  cp variants/_C_v$v.so tensorflow_distributed_amd/_C.so || exit 1
  timeout -k 10 200 python scripts/debug/gemm_probe.py --only wgrad --torch 0 > gpurun_out/wd_p$v.log 2>&1 || { echo "v$v probe failed"; tail -20 gpurun_out/wd_p$v.log; exit 1; }
  grep -v "dense4096\|amdgpu.ids" gpurun_out/wd_p$v.log | sed "s/^/v$v /" | sed 's/| torch.*//'
done
