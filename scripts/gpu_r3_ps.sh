#!/bin/bash
# GPU parameter server: unit (sync accumulator vs host optimizer) + launcher (async / backup) + speedup.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ps_gpu.py tests/test_runner_gpu.py -x -v -s --timeout 400 --timeout-method thread > gpurun_out/pytest_ps.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|worker step median|passed|failed" gpurun_out/pytest_ps.log | tail -20
[ $rc -ne 0 ] && tail -80 gpurun_out/pytest_ps.log
exit $rc
