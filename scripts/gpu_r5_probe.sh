#!/bin/bash
# Round 5: roofline floors (optimizer byte floor, launch boundary) + ResNet oracle rel-L2 calibration
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/debug/roofline_probe.py > gpurun_out/r5_roofline_probe.log 2>&1 || { tail -20 gpurun_out/r5_roofline_probe.log; exit 1; }
cat gpurun_out/r5_roofline_probe.log
timeout -k 10 600 python scripts/debug/resnet_oracle_rel.py > gpurun_out/r5_resnet_oracle_rel.log 2>&1 || { tail -20 gpurun_out/r5_resnet_oracle_rel.log; exit 1; }
cat gpurun_out/r5_resnet_oracle_rel.log
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -x -v --timeout 200 --timeout-method thread -k "captured_graph_keeps or rccl_bucketed or slot_mode" > gpurun_out/r5_probe_pytest.log 2>&1 || { tail -30 gpurun_out/r5_probe_pytest.log; exit 1; }
tail -3 gpurun_out/r5_probe_pytest.log
