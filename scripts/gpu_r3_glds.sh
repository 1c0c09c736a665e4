#!/bin/bash
# conv2 dgrad weight staging by LDS-DMA: engine tests, interleaved A/B, kernel table.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TEST_LIBS="base" TEST_FILES="tests/test_mnist_engine_gpu.py tests/test_dropout_curve_gpu.py" ROUNDS=3 TAG=glds ARMS="base|base|;nogl|nogl|" PROF=1 bash scripts/gpu_ab3.sh
