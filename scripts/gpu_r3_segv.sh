#!/bin/bash
# Isolate the ResNet forced-DP RCCL graph-replay segfault seen in the full GPU suite.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_resnet_gpu.py -k rccl_bucketed -v --timeout 120 --timeout-method thread > gpurun_out/segv_alone.log 2>&1; echo "alone rc=$?"; grep -E "PASS|FAIL|Fatal|passed|failed" gpurun_out/segv_alone.log | head
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/segv_file.log 2>&1; echo "file rc=$?"; grep -E "PASS|FAIL|Fatal|passed|failed" gpurun_out/segv_file.log | tail -30
