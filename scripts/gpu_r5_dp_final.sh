#!/bin/bash
# Round 5: DP tests, then forced-DP world-1 kernel tables / timelines (sfb+zero+mr, sfb+mr) and
# 1000-step bench lines interleaved with the fused one-GPU step.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dp_transport_gpu.py tests/test_graph_topology_gpu.py tests/test_ipc_gpu.py tests/test_mnist_engine_gpu.py > gpurun_out/r5_dpf_t.log 2>&1 || { tail -40 gpurun_out/r5_dpf_t.log; exit 1; }
tail -1 gpurun_out/r5_dpf_t.log
for sch in sfb+zero+mr sfb+mr; do
  rm -rf gpurun_out/r5_prof_dpf
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_prof_dpf -o run -- python3 bench.py --force_dp 1 --schedule $sch --steps 300 --warmup 20 --phases 0 --min_warmup_ms 0 --state_steps 0 > gpurun_out/r5_prof_dpf.log 2>&1 || { tail gpurun_out/r5_prof_dpf.log; exit 1; }
  db=$(find gpurun_out/r5_prof_dpf -name "*.db" | head -1)
  echo "## $sch: kernel table"
  python scripts/prof_summary.py $db --min-calls 100
  echo "## $sch: per-step timeline"
  python scripts/prof_timeline.py $db --anchor adam | tail -12
done
rm -rf gpurun_out/r5_prof_dpf
for r in 1 2 3; do
  for sch in sfb+zero+mr sfb+mr; do
    timeout -k 10 120 python bench.py --force_dp 1 --schedule $sch --steps 1000 --warmup 100 > gpurun_out/r5_dpf.log 2>&1 || { tail -5 gpurun_out/r5_dpf.log; exit 1; }
    echo "run $r forced-DP $sch: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_dpf.log)"
  done
  timeout -k 10 120 python bench.py --steps 1000 --warmup 100 > gpurun_out/r5_dpf.log 2>&1 || { tail -5 gpurun_out/r5_dpf.log; exit 1; }
  echo "run $r one-GPU fused step: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_dpf.log)"
done
