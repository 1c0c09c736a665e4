#!/bin/bash
# wgrad split-policy variants: probe wgrad per shape, then ResNet-50 ms/step, 2 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/tensorflow_distributed_amd
for lib in ${LIBS:-_C _C_px1k _C_px512 _C_px1kb1k}; do
  TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 200 python scripts/debug/gemm_probe.py --only wgrad --torch 0 > gpurun_out/probe_ws_$lib.log 2>&1 || { echo "probe $lib failed"; tail -5 gpurun_out/probe_ws_$lib.log; exit 1; }
done
paste <(grep wgrad gpurun_out/probe_ws__C.log | awk '{print $1, $4}') <(grep wgrad gpurun_out/probe_ws__C_px1k.log | awk '{print $4}') <(grep wgrad gpurun_out/probe_ws__C_px512.log | awk '{print $4}') <(grep wgrad gpurun_out/probe_ws__C_px1kb1k.log | awk '{print $4}')
for rep in 1 2; do
  for lib in ${LIBS:-_C _C_px1k _C_px512 _C_px1kb1k}; do
    TFD_NATIVE_LIB=$L/$lib.so timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 10 --warmup 3 > gpurun_out/rab_ws.log 2>&1 || { echo "bench $lib failed"; tail -20 gpurun_out/rab_ws.log; exit 1; }
    echo "$rep $lib: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rab_ws.log | head -1)"
  done
done
