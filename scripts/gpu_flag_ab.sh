#!/bin/bash
# bench.py flag A/B (ARMS="name:flags;..."), 1000/100 steps, interleaved rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
IFS=';' read -ra A <<< "${ARMS:-base:}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for arm in "${A[@]}"; do
    name=${arm%%:*}; flags=${arm#*:}
    timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --phases 0 $flags > gpurun_out/fab.log 2>&1 || { echo "bench $name failed"; tail -20 gpurun_out/fab.log; exit 1; }
    echo "$r $name: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fab.log)" | tee -a gpurun_out/flag_ab.log
  done
done
