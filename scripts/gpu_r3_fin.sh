#!/bin/bash
# ResNet: bn_final with 8 / 32 / 4 channels per block -- tests, interleaved ResNet-50 b128 A/B, kernel table
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/tensorflow_distributed_amd
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py tests/test_conv_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fin.log 2>&1 \
  || { echo "resnet tests failed"; tail -40 gpurun_out/pytest_fin.log; exit 1; }
echo "resnet tests: $(tail -1 gpurun_out/pytest_fin.log)"
for r in 1 2 3; do
  for arm in base fin32 fin4; do
    if [ $arm = base ]; then lib=$L/_C.so; else lib=$L/_C_$arm.so; fi
    TFD_NATIVE_LIB=$lib timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/fin.tmp 2>&1 \
      || { echo "bench failed"; tail -20 gpurun_out/fin.tmp; exit 1; }
    echo "$arm $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fin.tmp) $(grep -o '"value": [0-9.]*' gpurun_out/fin.tmp)" | tee -a gpurun_out/ab_fin.log
  done
done
rm -rf gpurun_out/prof_fin
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fin -o run -- python3 bench_resnet.py --depth 50 --batch_size 128 --steps 10 --warmup 3 > gpurun_out/prof_fin.log 2>&1 \
  || { echo "rocprof failed"; tail -20 gpurun_out/prof_fin.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof_fin -name "*.db" | head -1) --min-calls 5 > gpurun_out/kernels_fin.txt 2>&1
grep -E "kernel|bn_final" gpurun_out/kernels_fin.txt
rm -rf gpurun_out/prof_fin
