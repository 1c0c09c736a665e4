#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dp_transport_gpu.py tests/test_ipc_gpu.py tests/test_mnist_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_dpser2.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_dpser2.log; exit 1; }
tail -1 gpurun_out/pytest_dpser2.log
for r in 1 2; do
  for cfg in "ser:--zero 0" "serZ:--zero 1" "ar:--fc_sfb 0"; do
    n=${cfg%%:*}; f=${cfg#*:}
    timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --force_dp 1 $f > gpurun_out/dps.log 2>&1 || { echo "bench $n failed"; tail gpurun_out/dps.log; exit 1; }
    echo "$r $n: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dps.log)"
  done
done
rm -rf gpurun_out/prof_ser
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ser -o run -- python3 bench.py --steps 200 --warmup 20 --phases 0 --force_dp 1 > gpurun_out/prof_ser.log 2>&1 && python scripts/prof_summary.py $(find gpurun_out/prof_ser -name "*.db" | head -1) --min-calls 100 > gpurun_out/kernels_ser.txt && cat gpurun_out/kernels_ser.txt
