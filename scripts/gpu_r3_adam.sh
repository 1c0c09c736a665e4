#!/bin/bash
# fc-region Adam grid / strides-per-lane sweep (interleaved 1000-step benches) + determinism recheck of the bench
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ROUNDS=3 TAG=adam PROF=0 ARMS="base|base|;fcb1600|fcb1600|;fcb2048|fcb2048|;fcb800u4|fcb800u4|" bash scripts/gpu_ab3.sh || exit 1
for r in 1 2 3 4; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --min_warmup_ms 0 > gpurun_out/det3.tmp 2>&1 || { cat gpurun_out/det3.tmp; exit 1; }
  echo "phases=1 run $r $(grep -o '# world.*' gpurun_out/det3.tmp)" | tee -a gpurun_out/det3.log
done
