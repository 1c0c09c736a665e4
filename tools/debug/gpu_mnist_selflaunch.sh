#!/bin/bash
# repeat the self-launched MNIST bench with schedule probes (fresh engine per probe, closed after it)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
for n in ${NS:-2 4}; do
  for i in $(seq 1 ${N:-8}); do
    timeout -k 10 200 python bench.py --gpus $n --steps 20 --warmup 5 --probe_steps 20 --probe_warmup 5 > gpurun_out/mnsl_${n}_$i.log 2>&1
    rc=$?
    echo "n=$n run $i rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mnsl_${n}_$i.log)"
    [ $rc -eq 124 -o $rc -eq 137 ] && exit 1
    [ $rc -ne 0 ] && grep -vE "^\s*$" gpurun_out/mnsl_${n}_$i.log | grep -A30 -E "Fatal Python|free\(\)|corrupted|Error" | head -40
  done
done
exit 0
