#!/bin/bash
# idle gap before the driver-style 20/5 timed region: current (lean_gap 0), lean gap, +2 ms idle
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2 3 4; do
  for arm in ${ARMS:-"old:--lean_gap 0" "lean:--lean_gap 1" "idle2ms:--lean_gap 1 --idle_us 2000"}; do
    name=${arm%%:*}; flags=${arm#*:}
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --phases 0 $flags > gpurun_out/gap.log 2>&1 || { echo "bench failed"; cat gpurun_out/gap.log; exit 1; }
    echo "r=$r $name $(grep -o '"ms_per_step": [0-9.]*, "gpu_event_ms_per_step": [0-9.]*' gpurun_out/gap.log)" | tee -a gpurun_out/gap_ab.log
  done
done
