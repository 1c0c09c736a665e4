#!/bin/bash
# Round 5: HEAD check after the weight-gradient XCD renumbering: conv + ResNet GPU tests, ResNet-50 b128 steps.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_ops_gpu.py tests/test_resnet_gpu.py > gpurun_out/wgc_t.log 2>&1 || { tail -30 gpurun_out/wgc_t.log; exit 1; }
tail -1 gpurun_out/wgc_t.log
for r in 1 2; do
  timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/wgc_b.log 2>&1 || { tail -5 gpurun_out/wgc_b.log; exit 1; }
  echo "run $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/wgc_b.log)"
done
