#!/bin/bash
# HIP runtime graph-launch knobs on the driver-style timed region (host launch / sync wait split)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2; do
  for cfg in "none" "DEBUG_HIP_GRAPH_BATCH_SIZE=8" "DEBUG_HIP_GRAPH_BATCH_SIZE=32" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"; do
    if [ "$cfg" = none ]; then envs=""; else envs="$cfg"; fi
    r=$(env $envs TFD_BENCH_DIAG=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 2>gpurun_out/ge.err | grep -o '"ms_per_step": [0-9.]*') || { echo "bench $cfg failed"; tail -3 gpurun_out/ge.err; exit 1; }
    d=$(grep -o "host launch [0-9.]* us, sync wait [0-9.]* us" gpurun_out/ge.err | head -1)
    echo "run $i | $cfg $r ($d)" | tee -a gpurun_out/r4_graphenv.log
  done
done
