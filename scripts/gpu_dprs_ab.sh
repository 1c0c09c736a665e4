#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/tensorflow_distributed_amd
TFD_NATIVE_LIB=$L/_C_dxrs2.so timeout -k 10 300 python -u -m pytest tests/test_dp_transport_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "forced_dp_world1" > gpurun_out/pt_dxrs.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/pt_dxrs.log; exit 1; }
tail -1 gpurun_out/pt_dxrs.log
for r in 1 2 3; do
  for lib in _C _C_dxrs2; do
    TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --phases 0 --force_dp 1 --zero 1 > gpurun_out/dprs.log 2>&1 || { echo "bench failed"; tail gpurun_out/dprs.log; exit 1; }
    echo "$r $lib forced-DP zero $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dprs.log)"
  done
done
