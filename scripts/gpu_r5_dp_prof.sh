#!/bin/bash
# Round 5: kernel tables + per-step traces of the one-GPU fused step and the forced-DP world-1 step
# (sfb+zero, sfb, allreduce) at HEAD, plus 1000-step bench lines for each.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=gpurun_out/r5_dp.log
: > $L
for cfg in "base:" "zero:--force_dp 1 --fc_sfb 1 --zero 1" "sfb:--force_dp 1 --fc_sfb 1 --zero 0" "ar:--force_dp 1 --fc_sfb 0 --zero 0"; do
  n=${cfg%%:*}; f=${cfg#*:}
  timeout -k 10 120 python bench.py --steps 1000 --warmup 100 $f > gpurun_out/r5_b_$n.log 2>&1 || { echo "bench $n failed"; tail gpurun_out/r5_b_$n.log; exit 1; }
  echo "$n: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_b_$n.log) $(grep -o '"phases_ms": {[^}]*}' gpurun_out/r5_b_$n.log)" | tee -a $L
done
for cfg in "base:" "zero:--force_dp 1 --fc_sfb 1 --zero 1" "sfb:--force_dp 1 --fc_sfb 1 --zero 0" "ar:--force_dp 1 --fc_sfb 0 --zero 0"; do
  n=${cfg%%:*}; f=${cfg#*:}
  rm -rf gpurun_out/r5_prof_$n
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_prof_$n -o run -- python3 bench.py --steps 300 --warmup 20 --phases 0 --min_warmup_ms 0 --state_steps 0 $f > gpurun_out/r5_prof_$n.log 2>&1 || { echo "rocprof $n failed"; tail gpurun_out/r5_prof_$n.log; exit 1; }
  db=$(find gpurun_out/r5_prof_$n -name "*.db" | head -1)
  python scripts/prof_summary.py $db --min-calls 100 > gpurun_out/r5_kernels_$n.txt
  echo "== $n" >> $L; cat gpurun_out/r5_kernels_$n.txt >> $L
done
