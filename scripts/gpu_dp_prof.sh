#!/bin/bash
# forced-DP world-1 rehearsal of the multi-GPU step: bench lines + per-kernel profile (sfb, sfb+zero)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in "sfb:--fc_sfb 1 --zero 0" "zero:--fc_sfb 1 --zero 1" "ar:--fc_sfb 0 --zero 0"; do
  n=${cfg%%:*}; f=${cfg#*:}
  timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --force_dp 1 $f > gpurun_out/dp_$n.log 2>&1 || { echo "bench $n failed"; tail gpurun_out/dp_$n.log; exit 1; }
  echo "$n: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dp_$n.log) $(grep -o '"phases_ms": {[^}]*}' gpurun_out/dp_$n.log)"
done
for cfg in "sfb:--fc_sfb 1 --zero 0" "zero:--fc_sfb 1 --zero 1"; do
  n=${cfg%%:*}; f=${cfg#*:}
  rm -rf gpurun_out/prof_dp_$n
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dp_$n -o run -- python3 bench.py --steps 200 --warmup 20 --phases 0 --force_dp 1 $f > gpurun_out/prof_dp_$n.log 2>&1 || { echo "rocprof $n failed"; tail gpurun_out/prof_dp_$n.log; exit 1; }
  python scripts/prof_summary.py $(find gpurun_out/prof_dp_$n -name "*.db" | head -1) --min-calls 100 > gpurun_out/kernels_dp_$n.txt
  echo "== $n"; cat gpurun_out/kernels_dp_$n.txt
done
