#!/bin/bash
# Round 5: ResNet-50 b128 with the halo tiles on stage 1 (default) vs off, interleaved x3.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=gpurun_out/r5_halo_ab.log
: > $L
for r in 1 2 3; do
  for h in 0 1; do
    timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 30 --warmup 5 --conv_halo $h > gpurun_out/fb.tmp 2>&1 || { tail -20 gpurun_out/fb.tmp; exit 1; }
    echo "run $r halo $h: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fb.tmp)" | tee -a $L
  done
done
