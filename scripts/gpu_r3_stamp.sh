#!/bin/bash
# phase clocks of conv12 / head / conv2 backward at HEAD (TFD_STAMP build)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TFD_NATIVE_LIB=$PWD/tensorflow_distributed_amd/_C_stamp.so timeout -k 10 200 python -u scripts/debug/stamps.py > gpurun_out/stamps_head.log 2>&1 || { tail -30 gpurun_out/stamps_head.log; exit 1; }
grep -v Warn gpurun_out/stamps_head.log
for r in 1 2; do
  timeout -k 10 240 python bench_resnet.py --depth 18 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/rn18.tmp 2>&1 || { tail -20 gpurun_out/rn18.tmp; exit 1; }
  echo "resnet18 b128: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rn18.tmp) $(grep -o '"value": [0-9.]*' gpurun_out/rn18.tmp)" | tee -a gpurun_out/rn18.log
done
