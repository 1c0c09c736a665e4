#!/bin/bash
# ResNet: wgrad min pixels per split 2048 / 1024 / 512 -- tests, interleaved ResNet-50 b128 A/B, kernel table
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/tensorflow_distributed_amd
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py tests/test_conv_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_mp.log 2>&1 \
  || { echo "resnet tests failed"; tail -40 gpurun_out/pytest_mp.log; exit 1; }
echo "resnet tests: $(tail -1 gpurun_out/pytest_mp.log)"
for r in 1 2 3; do
  for arm in base mp1024 mp512; do
    if [ $arm = base ]; then lib=$L/_C.so; else lib=$L/_C_$arm.so; fi
    TFD_NATIVE_LIB=$lib timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/mp.tmp 2>&1 \
      || { echo "bench failed"; tail -20 gpurun_out/mp.tmp; exit 1; }
    echo "$arm $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mp.tmp) $(grep -o '"value": [0-9.]*' gpurun_out/mp.tmp)" | tee -a gpurun_out/ab_mp.log
  done
done
rm -rf gpurun_out/prof_mp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mp -o run -- python3 bench_resnet.py --depth 50 --batch_size 128 --steps 10 --warmup 3 > gpurun_out/prof_mp.log 2>&1 \
  || { echo "rocprof failed"; tail -20 gpurun_out/prof_mp.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof_mp -name "*.db" | head -1) --min-calls 5 > gpurun_out/kernels_mp.txt 2>&1
grep -E "kernel|bn_mpal" gpurun_out/kernels_mp.txt
rm -rf gpurun_out/prof_mp
