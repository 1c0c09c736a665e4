#!/bin/bash
# Timed-region sweep of --graph_steps at the driver's 20/5 (host wall vs GPU events), 3 interleaved rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/gsteps.log
: > $out
for r in 1 2 3; do
  for g in 1 5 10 20; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --graph_steps $g --phases 0 > gpurun_out/gs.json 2>/dev/null || { echo "bench failed g=$g"; exit 1; }
    echo "r=$r g=$g $(grep -o '"ms_per_step": [0-9.]*, "gpu_event_ms_per_step": [0-9.]*' gpurun_out/gs.json)" | tee -a $out
  done
done
