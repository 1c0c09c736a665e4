#!/bin/bash
# conv2 wgrad dz2 image: unpadded + chunk-swizzled (conflict-free B reads) vs pitch 72
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TEST_LIBS="base" TEST_FILES="tests/test_mnist_engine_gpu.py" ROUNDS=3 TAG=dzs ARMS="base|base|;noswzb|noswzb|" PROF=0 bash scripts/gpu_ab3.sh
