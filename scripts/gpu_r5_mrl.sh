#!/bin/bash
# Round 5: block order inside the merged DP tail launch (reduce blocks first vs last), forced-DP world 1.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=gpurun_out/r5_mrl.log
: > $L
for r in 1 2 3; do
  for sch in sfb+zero+mr sfb+mr; do
    for last in 0 1; do
      timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --force_dp 1 --schedule $sch --merge_reduce_last $last > gpurun_out/fb.tmp 2>&1 || { tail gpurun_out/fb.tmp; exit 1; }
      echo "run $r $sch last=$last: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fb.tmp)" | tee -a $L
    done
  done
done
