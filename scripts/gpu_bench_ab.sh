#!/bin/bash
# Interleaved A/B of bench.py argument sets on one lease: ARGS_A / ARGS_B, REPS rounds, 20/5 and 1000/100.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in $(seq 1 ${REPS:-2}); do
  for v in A B; do
    eval "args=\$ARGS_$v"
    for sw in "20 5" "1000 100"; do
      set -- $sw
      timeout -k 10 120 python bench.py --steps $1 --warmup $2 $args > gpurun_out/ab.log 2>&1 || { echo "bench failed"; cat gpurun_out/ab.log; exit 1; }
      echo "$v [$args] $1/$2: $(grep -o 'ms_per_step": [0-9.]*' gpurun_out/ab.log)"
    done
  done
done
