#!/bin/bash
# repeat the 2-rank self-launched ResNet bench with schedule probes; Python faulthandler traceback on abort
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
for i in $(seq 1 ${N:-14}); do
  timeout -k 10 200 python bench_resnet.py --gpus 2 --depth 18 --batch_size 8 --image 64 --steps 3 --warmup 1 \
    --bucket_candidates 0.5,2 --probe_steps 3 --probe_warmup 1 ${EXTRA} > gpurun_out/rnsl_$i.log 2>&1
  rc=$?
  echo "run $i rc=$rc"
  [ $rc -eq 124 -o $rc -eq 137 ] && exit 1
  [ $rc -ne 0 ] && grep -vE "^\s*$" gpurun_out/rnsl_$i.log | grep -A40 -E "Fatal Python|free\(\)|corrupted" | head -60
done
exit 0
