#!/bin/bash
# fused conv2 wgrad + dgrad blocks (dgrad weights' LDS-DMA under the wgrad's last image): engine tests,
# interleaved A/B, kernel table, phase clocks.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TEST_LIBS="base" TEST_FILES="tests/test_mnist_engine_gpu.py tests/test_dropout_curve_gpu.py" ROUNDS=3 TAG=fu ARMS="base|base|;nofu|nofu|" PROF=1 bash scripts/gpu_ab3.sh || exit 1
TFD_NATIVE_LIB=$PWD/tensorflow_distributed_amd/_C_stamp.so timeout -k 10 200 python scripts/debug/stamps.py > gpurun_out/stamps_fu.log 2>&1; echo "stamps rc=$?"; tail -15 gpurun_out/stamps_fu.log
