#!/bin/bash
# driver-style timed region (--steps 20 --warmup 5): steps per captured graph 20 (one launch) vs 5 vs 1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2 3 4; do
  line="run $i"
  for gs in 20 5 1; do
    r=$(TFD_BENCH_DIAG=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --graph_steps $gs 2>gpurun_out/gs.err | grep -o '"ms_per_step": [0-9.]*') || { echo "bench gs=$gs failed"; cat gpurun_out/gs.err | tail -5; exit 1; }
    d=$(grep -o "host launch [0-9.]* us, sync wait [0-9.]* us" gpurun_out/gs.err | head -1)
    line="$line | gs$gs $r ($d)"
  done
  echo "$line" | tee -a gpurun_out/r4_gsteps.log
done
