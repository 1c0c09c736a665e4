#!/bin/bash
# phase clocks of conv12 / head / conv2 backward at HEAD (TFD_STAMP build)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TFD_NATIVE_LIB=$PWD/tensorflow_distributed_amd/_C_stamp.so timeout -k 10 200 python -u scripts/debug/stamps.py > gpurun_out/stamps_head.log 2>&1 || { tail -30 gpurun_out/stamps_head.log; exit 1; }
grep -v Warn gpurun_out/stamps_head.log
