#!/bin/bash
# Round 5: halo-tile 3x3 convs: numerics (conv op tests on every path), per-layer probe vs the gather.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv_ops_gpu.py -x -q --timeout 200 --timeout-method thread -k "halo" > gpurun_out/r5_halo_pytest.log 2>&1 || { tail -40 gpurun_out/r5_halo_pytest.log; exit 1; }
tail -2 gpurun_out/r5_halo_pytest.log
timeout -k 10 300 python scripts/debug/halo_probe.py > gpurun_out/r5_halo_probe.log 2>&1 || { tail -20 gpurun_out/r5_halo_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5_halo_probe.log
