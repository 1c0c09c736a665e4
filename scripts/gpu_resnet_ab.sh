#!/bin/bash
# ResNet-50 b128 A/B of one bench_resnet.py switch (alternating, same box) + rocprofv3 of the B side.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-rab}; FLAG=${FLAG:---fuse_joins}
for v in 0 1 0 1; do
  timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 30 --warmup 5 $FLAG $v > gpurun_out/bench_${TAG}_$v.log 2>&1 \
    || { echo "bench failed"; tail -30 gpurun_out/bench_${TAG}_$v.log; exit 1; }
  echo "$FLAG=$v: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_${TAG}_$v.log)"
done
rm -rf gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench_resnet.py --depth 50 --batch_size 128 --steps 3 --warmup 1 $FLAG 1 \
  > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof_$TAG -name "*.db" | head -1) --min-calls 3 > gpurun_out/kernels_$TAG.txt
head -24 gpurun_out/kernels_$TAG.txt
