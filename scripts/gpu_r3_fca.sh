#!/bin/bash
# one-GPU fc1 Adam in the dW epilogue: engine tests, interleaved A/B (--fc_adam 1/0), kernel table +
# per-step timeline.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mnist_engine_gpu.py tests/test_dropout_curve_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fca.log 2>&1 \
  || { echo "engine tests failed"; tail -40 gpurun_out/pytest_fca.log; exit 1; }
echo "engine tests: $(tail -1 gpurun_out/pytest_fca.log)"
ROUNDS=3 TAG=fca ARMS="${ARMS:-fca|base|;nofca|base|--fc_adam 0}" bash scripts/gpu_ab3.sh || exit 1
SUITE=0 bash scripts/gpu_r3_tl.sh
