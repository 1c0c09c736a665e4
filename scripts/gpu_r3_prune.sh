#!/bin/bash
# After pruning the losing schedule knobs: engine + DP suites, driver-style bench.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mnist_engine_gpu.py tests/test_dp_transport_gpu.py tests/test_ipc_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_prune.log 2>&1 || { echo "pytest failed: $?"; grep -E "FAILED|ERROR" gpurun_out/pytest_prune.log | head; tail -60 gpurun_out/pytest_prune.log; exit 1; }
tail -2 gpurun_out/pytest_prune.log
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_drv.log 2>&1 && tail -1 gpurun_out/bench_drv.log | cut -c1-200
