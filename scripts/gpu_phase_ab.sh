#!/bin/bash
# strided-dgrad phase decomposition A/B: conv + ResNet tests, probe of the stride-2 shapes (dgrad), ResNet-50 arms
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/tensorflow_distributed_amd
timeout -k 10 600 python -u -m pytest tests/test_conv_ops_gpu.py tests/test_resnet_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_ph.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_ph.log; exit 1; }
tail -1 gpurun_out/pytest_ph.log
for lib in _C _C_nophase; do
  TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 200 python scripts/debug/gemm_probe.py --only dgrad --match s2 --torch 1 > gpurun_out/probe_ph_$lib.log 2>&1 || { echo "probe $lib failed"; tail -20 gpurun_out/probe_ph_$lib.log; exit 1; }
  echo "== $lib"; grep dgrad gpurun_out/probe_ph_$lib.log
done
for rep in 1 2; do
  for lib in _C_nophase _C; do
    TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 10 --warmup 3 > gpurun_out/rab_ph_$lib.log 2>&1 || { echo "bench $lib failed"; tail -20 gpurun_out/rab_ph_$lib.log; exit 1; }
    echo "$rep $lib: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rab_ph_$lib.log | head -1)"
  done
done
