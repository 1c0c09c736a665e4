#!/bin/bash
# ResNet-50 b128 kernel table at HEAD (args after the script go to bench_resnet.py)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_rn
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run -- python3 bench_resnet.py --depth 50 --batch_size 128 --steps 10 --warmup 3 "$@" > gpurun_out/prof_rn.log 2>&1 || { tail -20 gpurun_out/prof_rn.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof_rn -name "*.db" | head -1) > gpurun_out/rn50_kernels_head.txt
rm -rf gpurun_out/prof_rn
