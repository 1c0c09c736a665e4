#!/bin/bash
# BN totals (last-arriver, no bn_final launch) A/B: conv + ResNet tests, ResNet-50 / -18 arms, kernel profile
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/tensorflow_distributed_amd
timeout -k 10 600 python -u -m pytest tests/test_conv_ops_gpu.py tests/test_resnet_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_bt.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" gpurun_out/pytest_bt.log | head; tail -40 gpurun_out/pytest_bt.log; exit 1; }
tail -1 gpurun_out/pytest_bt.log
for rep in 1 2; do
  for arm in ${ARMS:-"_C_nototals:1" "_C:1"}; do
    lib=${arm%%:*}; bits=${arm#*:}
    for d in 50 18; do
      TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 300 python bench_resnet.py --depth $d --batch_size 128 --steps 10 --warmup 3 --relu_bits $bits > gpurun_out/rab_bt.log 2>&1 || { echo "bench $lib failed"; tail -20 gpurun_out/rab_bt.log; exit 1; }
      echo "$rep $lib bits=$bits r$d: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rab_bt.log | head -1)"
    done
  done
done
rm -rf gpurun_out/prof_bt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bt -o run -- python3 bench_resnet.py --depth 50 --batch_size 128 --steps 6 --warmup 2 > gpurun_out/prof_bt.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_bt.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof_bt -name "*.db" | head -1) --min-calls 6 > gpurun_out/kernels_bt.txt
head -24 gpurun_out/kernels_bt.txt
