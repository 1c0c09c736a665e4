#!/bin/bash
# LDS-staged conv epilogue A/B: conv/ResNet GPU tests on the new lib, GEMM probe (fwd/dgrad) on the
# new and ref libs, then ResNet-50 b128 arms (lib:flags), 2 interleaved rounds.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-epi}
L=$PWD/tensorflow_distributed_amd
timeout -k 10 600 python -u -m pytest tests/test_conv_ops_gpu.py tests/test_resnet_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
for lib in _C _C_ref; do
  TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 200 python scripts/debug/gemm_probe.py --only fwd,dgrad --torch 0 > gpurun_out/probe_${TAG}_$lib.log 2>&1 || { echo "probe $lib failed"; tail -20 gpurun_out/probe_${TAG}_$lib.log; exit 1; }
  echo "$lib: $(grep TOTAL gpurun_out/probe_${TAG}_$lib.log | tr '\n' ' ')"
done
IFS=';' read -ra ARMS <<< "${ARMS:-ref:_C_ref:--fuse_joins 0;new:_C:--fuse_joins 0;newjoin:_C:--fuse_joins 1}"
for rep in 1 2; do
  for arm in "${ARMS[@]}"; do
    IFS=':' read -r name lib flags <<< "$arm"
    TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 300 python bench_resnet.py --depth ${DEPTH:-50} --batch_size 128 --steps 10 --warmup 3 $flags > gpurun_out/rab_${TAG}_$name.log 2>&1 || { echo "bench $name failed"; tail -20 gpurun_out/rab_${TAG}_$name.log; exit 1; }
    echo "$rep $name: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rab_${TAG}_$name.log | head -1)"
  done
done
