#!/bin/bash
# Round 5: ResNet-50 b128 bench, backward on the caller's thread (HEAD) vs the autograd device
# thread (TFD_RN_MT_BACKWARD=1, this A/B only), interleaved.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for mt in 0 1; do
    TFD_RN_MT_BACKWARD=$mt timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/r5_rnab.log 2>&1 || { tail -20 gpurun_out/r5_rnab.log; exit 1; }
    echo "run $r mt_backward=$mt: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_rnab.log)"
  done
done
