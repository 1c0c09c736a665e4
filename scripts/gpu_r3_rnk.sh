#!/bin/bash
# ResNet-50 b128 kernel table at HEAD
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_rnk
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rnk -o run -- python3 bench_resnet.py --depth 50 --batch_size 128 --steps 10 --warmup 3 > gpurun_out/prof_rnk.log 2>&1 \
  || { echo "rocprof failed"; tail -20 gpurun_out/prof_rnk.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof_rnk -name "*.db" | head -1) --min-calls 5 > gpurun_out/kernels_rnk.txt 2>&1
head -16 gpurun_out/kernels_rnk.txt
rm -rf gpurun_out/prof_rnk
