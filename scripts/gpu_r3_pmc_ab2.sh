#!/bin/bash
# PMC passes at HEAD (derived per-kernel table) + conv2 wgrad 4 images x 8 tap groups A/B.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash scripts/gpu_pmc.sh > gpurun_out/pmc_all.txt 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_all.txt; exit 1; }
python scripts/pmc_derived.py gpurun_out/pmc_all.txt > gpurun_out/pmc_derived.txt 2>&1; cat gpurun_out/pmc_derived.txt
TEST_LIBS="c2w48" TEST_FILES=tests/test_mnist_engine_gpu.py ROUNDS=3 TAG=c2w48 ARMS="base|base|;c2w48|c2w48|" bash scripts/gpu_ab3.sh
