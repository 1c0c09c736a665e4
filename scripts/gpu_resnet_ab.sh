#!/bin/bash
# ResNet A/B: conv/BN/ResNet GPU tests, then bench_resnet.py for each ARM ("name:flags;...")
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-rab}
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_conv_ops_gpu.py tests/test_resnet_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error" gpurun_out/pytest_$TAG.log | tail -30; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
  grep -E "passed|failed" gpurun_out/pytest_$TAG.log | tail -2
fi
IFS=';' read -ra ARMS <<< "${ARMS:-base:--bn_stats 0;stats:--bn_stats 1}"
for rep in 1 2; do
  for arm in "${ARMS[@]}"; do
    name=${arm%%:*}; flags=${arm#*:}
    lib=$PWD/tensorflow_distributed_amd/_C_${name}.so; [ -f "$lib" ] || lib=$PWD/tensorflow_distributed_amd/_C.so
    TFD_NATIVE_LIB=$lib timeout -k 10 300 python bench_resnet.py --depth ${DEPTH:-50} --batch_size 128 --steps 10 --warmup 3 $flags > gpurun_out/rab_${TAG}_$name.log 2>&1 || { echo "bench $name failed"; tail -20 gpurun_out/rab_${TAG}_$name.log; exit 1; }
    echo "$rep $name: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rab_${TAG}_$name.log | head -1)"
  done
done
if [ "${PROF:-0}" = "1" ]; then
  rm -rf gpurun_out/prof_$TAG
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench_resnet.py --depth ${DEPTH:-50} --batch_size 128 --steps 3 --warmup 1 > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
  python scripts/prof_summary.py $(find gpurun_out/prof_$TAG -name "*.db" | head -1) --min-calls 3 > gpurun_out/kernels_$TAG.txt
  head -25 gpurun_out/kernels_$TAG.txt
fi
