#!/bin/bash
# serialized vs overlapped SFB DP schedule: DP tests, then the world-1 rehearsal A/B (1000/100), 2 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dp_transport_gpu.py tests/test_ipc_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_dpser.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_dpser.log; exit 1; }
tail -1 gpurun_out/pytest_dpser.log
for r in 1 2; do
  for cfg in "ser:--dp_serial 1 --zero 0" "ovl:--dp_serial 0 --zero 0" "serZ:--dp_serial 1 --zero 1" "ovlZ:--dp_serial 0 --zero 1"; do
    n=${cfg%%:*}; f=${cfg#*:}
    timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --force_dp 1 --fc_sfb 1 $f > gpurun_out/dps.log 2>&1 || { echo "bench $n failed"; tail gpurun_out/dps.log; exit 1; }
    echo "$r $n: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dps.log) $(grep -o '"phases_ms": {[^}]*}' gpurun_out/dps.log)"
  done
done
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 200 --warmup 20 > gpurun_out/dps2.log 2>&1 && grep -o '"ms_per_step": [0-9.]*' gpurun_out/dps2.log
