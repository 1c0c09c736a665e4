#!/bin/bash
# ResNet-50 b128 kernel tables in row mode (--bn_slots 0) and slot mode (4)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for sl in 0 4; do
  rm -rf gpurun_out/prof_sl$sl
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sl$sl -o run -- python3 bench_resnet.py --depth 50 --batch_size 128 --steps 10 --warmup 3 --bn_slots $sl > gpurun_out/prof_sl$sl.log 2>&1 || { tail -20 gpurun_out/prof_sl$sl.log; exit 1; }
  python scripts/prof_summary.py $(find gpurun_out/prof_sl$sl -name "*.db" | head -1) > gpurun_out/rn50_kernels_sl$sl.txt
  rm -rf gpurun_out/prof_sl$sl
done
