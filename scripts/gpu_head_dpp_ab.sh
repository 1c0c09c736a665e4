#!/bin/bash
# head kernel: logits wave sums by DPP (TFD_HEAD_DPP) -- phase clocks, engine numerics tests, bench A/B
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TFD_NATIVE_LIB=$PWD/tensorflow_distributed_amd/_C_stamphd.so timeout -k 10 120 python scripts/debug/stamps.py > gpurun_out/stamps_stamphd.log 2>&1 \
  || { echo "stamps failed"; tail -20 gpurun_out/stamps_stamphd.log; exit 1; }
grep head gpurun_out/stamps_stamphd.log
TAG=hdpp VARIANTS="base hdpp" bash scripts/gpu_variant_ab.sh
