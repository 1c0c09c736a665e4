#!/bin/bash
# Round 5: driver-style timed region (--steps 20 --warmup 5) with --lead_steps 0 / 2 / 4 interleaved.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2 3 4; do
  for L in 0 2 4; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --lead_steps $L > gpurun_out/r5_lead.log 2>&1 || { tail -5 gpurun_out/r5_lead.log; exit 1; }
    echo "run $r lead=$L: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_lead.log) $(grep -o '"gpu_event_ms_per_step": [0-9.]*' gpurun_out/r5_lead.log)"
  done
done
