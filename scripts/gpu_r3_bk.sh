#!/bin/bash
# fc1 dX K-tile 256 (4 K-steps) vs 128 (8): one GPU and the DP rehearsal (dX-alone tiles)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TEST_LIBS="bk256" ROUNDS=3 TAG=bk PROF=1 ARMS="bk256|bk256|;base|base|;dp_bk256|bk256|--force_dp 1;dp_base|base|--force_dp 1" bash scripts/gpu_ab3.sh
