#!/bin/bash
# masked identity-shortcut join: ResNet GPU tests, then interleaved ResNet-50 b128 A/B (masked_join 0 / 1)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_resnet_gpu.py \
  > gpurun_out/r4_mj_tests.log 2>&1 || { tail -30 gpurun_out/r4_mj_tests.log; exit 1; }
tail -3 gpurun_out/r4_mj_tests.log
for i in 1 2 3; do
  line="run $i"
  for mj in 0 1; do
    r=$(timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 --masked_join $mj 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || { echo "bench mj=$mj failed"; exit 1; }
    line="$line | mj$mj $r"
  done
  echo "$line" | tee -a gpurun_out/r4_mj_ab.log
done
