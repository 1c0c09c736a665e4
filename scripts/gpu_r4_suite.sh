#!/bin/bash
# full GPU suite + smoke at HEAD
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_suite.log 2>&1 \
  || { echo "gpu suite failed"; grep -E "FAILED|Error|error" gpurun_out/pytest_gpu_suite.log | head -20; tail -30 gpurun_out/pytest_gpu_suite.log; exit 1; }
echo "gpu suite: $(tail -1 gpurun_out/pytest_gpu_suite.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
