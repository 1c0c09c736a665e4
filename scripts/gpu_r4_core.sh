#!/bin/bash
# 256-row core in the conv ops: numerics on both cores, per-layer probe, ResNet-50 with each core mode.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv_ops_gpu.py tests/test_resnet_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_core_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r4_core_tests.log | head -20; tail -30 gpurun_out/r4_core_tests.log; exit 1; }
tail -1 gpurun_out/r4_core_tests.log
timeout -k 10 300 python scripts/debug/gemm_probe.py --iters 10 > gpurun_out/r4_probe.log 2>&1 || { tail -20 gpurun_out/r4_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4_probe.log | tail -64
for m in 0 1 2; do
  TFD_G256=$m timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/r4_rn50_$m.log 2>&1 || { tail -20 gpurun_out/r4_rn50_$m.log; exit 1; }
  echo "TFD_G256=$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4_rn50_$m.log)"
done
