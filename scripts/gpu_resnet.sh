#!/bin/bash
# ResNet bench (1 GPU) + rocprofv3 kernel summary.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-r}
ARGS=${ARGS:---depth 50 --batch_size 64 --steps 10 --warmup 3}
timeout -k 10 600 python bench_resnet.py $ARGS > gpurun_out/bench_resnet_$TAG.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_resnet_$TAG.log; exit 1; }
cat gpurun_out/bench_resnet_$TAG.log
if [ "${PROF:-1}" = "1" ]; then
  rm -rf gpurun_out/prof_resnet_$TAG
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet_$TAG -o run -- python3 bench_resnet.py $ARGS --steps 3 --warmup 1 > gpurun_out/prof_resnet_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_resnet_$TAG.log; exit 1; }
  python scripts/prof_summary.py $(find gpurun_out/prof_resnet_$TAG -name "*.db" | head -1) --min-calls 3 > gpurun_out/kernels_resnet_$TAG.txt
  head -30 gpurun_out/kernels_resnet_$TAG.txt
fi
