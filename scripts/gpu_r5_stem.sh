#!/bin/bash
# Round 5: the width-paired ResNet stem: conv + ResNet GPU tests, stem probe, then ResNet-50 / -18 b128
# with the paired stem (--stem_w2 1, HEAD) vs the channel-padded one (0), 3 interleaved rounds.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_ops_gpu.py tests/test_resnet_gpu.py > gpurun_out/stem_t.log 2>&1 || { tail -30 gpurun_out/stem_t.log; exit 1; }
tail -1 gpurun_out/stem_t.log
for r in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 --stem_w2 $v > gpurun_out/stem_b$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/stem_b$v.log; exit 1; }
    timeout -k 10 300 python bench_resnet.py --depth 18 --batch_size 128 --steps 20 --warmup 5 --stem_w2 $v > gpurun_out/stem_c$v.log 2>&1 || { echo "r18 bench $v failed"; tail -5 gpurun_out/stem_c$v.log; exit 1; }
    echo "run $r stem_w2=$v: r50 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/stem_b$v.log) r18 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/stem_c$v.log)"
  done
done
