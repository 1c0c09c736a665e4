#!/bin/bash
# fused stem bn+relu+maxpool: op + ResNet tests, interleaved ResNet-50 b128 A/B (--fuse_stem_pool 0/1)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_ops_gpu.py -k "maxpool or batchnorm" && timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_resnet_gpu.py > gpurun_out/r4_stem_tests.log 2>&1 \
  || { tail -30 gpurun_out/r4_stem_tests.log; exit 1; }
tail -1 gpurun_out/r4_stem_tests.log
for i in 1 2 3; do
  line="run $i"
  for f in 0 1; do
    r=$(timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 --fuse_stem_pool $f 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || { echo "bench fuse=$f failed"; exit 1; }
    line="$line | stem$f $r"
  done
  echo "$line" | tee -a gpurun_out/r4_stem_ab.log
done
