#!/bin/bash
# BN statistics slot mode: conv-op + ResNet GPU tests, interleaved ResNet-50 b128 A/B over --bn_slots,
# kernel tables of row mode / slot mode
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_ops_gpu.py tests/test_resnet_gpu.py \
  > gpurun_out/r4_slots_tests.log 2>&1 || { tail -40 gpurun_out/r4_slots_tests.log; exit 1; }
tail -3 gpurun_out/r4_slots_tests.log
for i in 1 2 3; do
  line="run $i"
  for sl in ${SLOTS:-0 4 16}; do
    r=$(timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 --bn_slots $sl 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || { echo "bench slots=$sl failed"; exit 1; }
    line="$line | s$sl $r"
  done
  echo "$line" | tee -a gpurun_out/r4_slots_ab.log
done
[ -n "$NOPROF" ] && exit 0
for sl in 0 4; do
  rm -rf gpurun_out/prof_sl$sl
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sl$sl -o run -- python3 bench_resnet.py --depth 50 --batch_size 128 --steps 10 --warmup 3 --bn_slots $sl > gpurun_out/prof_sl$sl.log 2>&1 || { tail -20 gpurun_out/prof_sl$sl.log; exit 1; }
  python scripts/prof_summary.py $(find gpurun_out/prof_sl$sl -name "*.db" | head -1) > gpurun_out/rn50_kernels_sl$sl.txt
  rm -rf gpurun_out/prof_sl$sl
done
