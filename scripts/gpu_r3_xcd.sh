#!/bin/bash
# fc1 dX tiles: XCD-grouped W1 column tiles vs round-robin
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TEST_LIBS="base" TEST_FILES="tests/test_mnist_engine_gpu.py tests/test_ipc_gpu.py" ROUNDS=3 TAG=xcd PROF=1 ARMS="base|base|;noxcd|noxcd|" bash scripts/gpu_ab3.sh
