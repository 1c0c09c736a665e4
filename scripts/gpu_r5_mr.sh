#!/bin/bash
# Round 5: merged DP tail (slab reduce inside the SFB GEMM launch): DP tests, 1000-step forced-DP
# world-1 bench lines per schedule (interleaved twice), kernel trace of the merged schedules.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=gpurun_out/r5_mr.log
: > $L
timeout -k 10 900 python -u -m pytest tests/test_dp_transport_gpu.py tests/test_graph_topology_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5_mr_pytest.log 2>&1 || { tail -40 gpurun_out/r5_mr_pytest.log; exit 1; }
tail -1 gpurun_out/r5_mr_pytest.log | tee -a $L
for r in 1 2; do
for n in sfb+zero+mr sfb+mr sfb+zero sfb; do
  timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --force_dp 1 --schedule $n > gpurun_out/r5_mr_b.log 2>&1 || { echo "bench $n failed"; tail gpurun_out/r5_mr_b.log; exit 1; }
  echo "$n: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_mr_b.log)" | tee -a $L
done
done
for n in sfb+zero+mr sfb+mr; do
  rm -rf gpurun_out/r5_prof_$n
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_prof_$n -o run -- python3 bench.py --steps 300 --warmup 20 --phases 0 --min_warmup_ms 0 --state_steps 0 --force_dp 1 --schedule $n > gpurun_out/r5_prof_$n.log 2>&1 || { echo "rocprof $n failed"; tail gpurun_out/r5_prof_$n.log; exit 1; }
  db=$(find gpurun_out/r5_prof_$n -name "*.db" | head -1)
  python scripts/prof_summary.py $db --min-calls 100 > gpurun_out/r5_kernels_$n.txt
  echo "== $n" >> $L; cat gpurun_out/r5_kernels_$n.txt >> $L
done
