#!/bin/bash
# Full GPU suite + smoke.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r4_suite.log 2>&1 \
  || { echo "suite failed"; grep -E "FAIL|Error" gpurun_out/r4_suite.log | tail -20; tail -50 gpurun_out/r4_suite.log; exit 1; }
tail -1 gpurun_out/r4_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
