#!/bin/bash
# wgrad tile A/B: conv tests on the new lib, GEMM probe (wgrad) new vs 64x64-only, ResNet-50 arms
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/tensorflow_distributed_amd
timeout -k 10 300 python -u -m pytest tests/test_conv_ops_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_wg.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_wg.log; exit 1; }
tail -1 gpurun_out/pytest_wg.log
for lib in _C _C_wg64; do
  TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 200 python scripts/debug/gemm_probe.py --only wgrad --torch 0 > gpurun_out/probe_wg_$lib.log 2>&1 || { echo "probe $lib failed"; tail -20 gpurun_out/probe_wg_$lib.log; exit 1; }
done
paste <(grep wgrad gpurun_out/probe_wg__C.log | awk '{print $1, $4}') <(grep wgrad gpurun_out/probe_wg__C_wg64.log | awk '{print $4}')
for rep in 1 2; do
  for lib in _C_wg64 _C; do
    TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 10 --warmup 3 > gpurun_out/rab_wg_$lib.log 2>&1 || { echo "bench $lib failed"; tail -20 gpurun_out/rab_wg_$lib.log; exit 1; }
    echo "$rep $lib: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rab_wg_$lib.log | head -1)"
  done
done
