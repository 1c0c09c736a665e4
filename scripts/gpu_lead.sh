#!/bin/bash
# timed-region lead-in A/B at the driver's 20/5: L one-step graphs, then one (20-L)-step graph
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2 3 4; do
  for L in ${LEADS:-0 2 3}; do
    TFD_BENCH_DIAG=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --phases 0 --lead_steps $L > gpurun_out/lead.log 2>&1 || { echo "bench failed"; cat gpurun_out/lead.log; exit 1; }
    echo "r=$r L=$L $(grep -o 'host launch [0-9.]* us' gpurun_out/lead.log) $(grep -o '"ms_per_step": [0-9.]*, "gpu_event_ms_per_step": [0-9.]*' gpurun_out/lead.log)" | tee -a gpurun_out/lead_sweep.log
  done
done
