#!/bin/bash
# conv1 X8 gather + one-launch conv2 backward: engine/oracle tests, interleaved A/B, kernel table +
# per-step timeline, then the full GPU suite.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mnist_engine_gpu.py tests/test_dropout_curve_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab1.log 2>&1 \
  || { echo "engine tests failed"; tail -40 gpurun_out/pytest_ab1.log; exit 1; }
echo "engine tests: $(tail -1 gpurun_out/pytest_ab1.log)"
ROUNDS=3 TAG=ab1 ARMS="${ARMS:-base|base|;nox8|nox8|;bwd2|bwd2|}" bash scripts/gpu_ab3.sh || exit 1
SUITE=${SUITE:-1} bash scripts/gpu_r3_tl.sh
