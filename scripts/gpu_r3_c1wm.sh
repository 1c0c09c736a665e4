#!/bin/bash
# conv1 weight gradient on the matrix core (dgrad tail): engine/oracle tests, interleaved A/B vs the
# VALU tail, dgrad phase clocks.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TEST_LIBS="base" TEST_FILES="tests/test_mnist_engine_gpu.py tests/test_dropout_curve_gpu.py" ROUNDS=3 TAG=c1wm ARMS="base|base|;c1wv|c1wv|" PROF=1 bash scripts/gpu_ab3.sh || exit 1
TFD_NATIVE_LIB=$PWD/tensorflow_distributed_amd/_C_stamp.so timeout -k 10 200 python scripts/debug/stamps.py > gpurun_out/stamps_c1wm.log 2>&1; echo "stamps rc=$?"; tail -9 gpurun_out/stamps_c1wm.log
