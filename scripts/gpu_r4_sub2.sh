#!/bin/bash
# stride-2 shortcut dgrad on its own grid: op + ResNet tests, interleaved ResNet-50 b128 A/B (TFD_JOIN_SUB2 0/1)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_ops_gpu.py -k "stride2 or dgrad" > gpurun_out/r4_sub2_tests.log 2>&1 \
  && timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_resnet_gpu.py >> gpurun_out/r4_sub2_tests.log 2>&1 \
  || { tail -30 gpurun_out/r4_sub2_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_sub2_tests.log
for i in 1 2 3; do
  line="run $i"
  for v in 0 1; do
    r=$(TFD_JOIN_SUB2=$v timeout -k 10 240 python bench_resnet.py --depth ${DEPTH:-50} --batch_size 128 --steps 20 --warmup 5 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || { echo "bench sub2=$v failed"; exit 1; }
    line="$line | sub2_$v $r"
  done
  echo "$line" | tee -a gpurun_out/r4_sub2_ab.log
done
