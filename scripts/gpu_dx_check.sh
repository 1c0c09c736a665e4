#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mnist_engine_gpu.py tests/test_dp_transport_gpu.py tests/test_ipc_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_dxc.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt_dxc.log; exit 1; }
tail -1 gpurun_out/pt_dxc.log
for r in 1 2; do
  timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --phases 0 > gpurun_out/dx.log 2>&1 && one=$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dx.log)
  timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --phases 0 --force_dp 1 --zero 1 > gpurun_out/dx.log 2>&1 && echo "$r one-GPU $one | forced-DP zero $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dx.log)"
  timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --phases 0 --force_dp 1 --zero 0 > gpurun_out/dx.log 2>&1 && echo "$r forced-DP sfb $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dx.log)"
done
