#!/bin/bash
# driver-style 20/5 timed region: blocking synchronize vs event polling before it, 4 interleaved rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2 3 4; do
  for sp in 0 1; do
    TFD_BENCH_DIAG=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --phases 0 --spin_sync $sp > gpurun_out/spin.log 2>&1 || { echo "bench failed"; cat gpurun_out/spin.log; exit 1; }
    echo "r=$r spin=$sp $(grep -o 'host launch.*barrier [0-9.]* us' gpurun_out/spin.log) $(grep -o '"ms_per_step": [0-9.]*, "gpu_event_ms_per_step": [0-9.]*' gpurun_out/spin.log)" | tee -a gpurun_out/spin_ab.log
  done
done
