#!/bin/bash
# head kernel: per-phase clocks (TFD_STAMP builds) with and without the early output-weight loads,
# then the interleaved bench A/B of the two libraries
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in stamp stamphp; do
  echo "== $v"
  TFD_NATIVE_LIB=$PWD/tensorflow_distributed_amd/_C_$v.so timeout -k 10 120 python scripts/debug/stamps.py > gpurun_out/stamps_$v.log 2>&1 \
    || { echo "stamps $v failed"; tail -20 gpurun_out/stamps_$v.log; exit 1; }
  grep head gpurun_out/stamps_$v.log
done
TAG=head VARIANTS="base hpref" bash scripts/gpu_variant_ab.sh
