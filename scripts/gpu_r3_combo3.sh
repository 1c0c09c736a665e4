#!/bin/bash
# GPU PS tests; deferred fc1 Adam (512-thread fused kernel) bit-identity + A/B; head phase clocks.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mnist_engine_gpu.py -k "captured or oracle" -q --timeout 120 --timeout-method thread > gpurun_out/pytest_defer.log 2>&1; rc=$?
echo "engine tests rc=$rc"; tail -2 gpurun_out/pytest_defer.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
ROUNDS=3 TAG=defer2 ARMS="base|base|;defer|base|--defer_fc1_adam 1" bash scripts/gpu_ab3.sh || exit 1
TFD_NATIVE_LIB=$PWD/tensorflow_distributed_amd/_C_stamp.so timeout -k 10 120 python scripts/debug/stamps.py > gpurun_out/stamps.log 2>&1; echo "stamps rc=$?"; tail -8 gpurun_out/stamps.log
bash scripts/gpu_r3_ps.sh
