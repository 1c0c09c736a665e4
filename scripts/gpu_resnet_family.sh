#!/bin/bash
# ResNet-18/50 benches at per-GPU batch 128 on one GPU, the same-hardware PyTorch (MIOpen) path for
# comparison, and a rocprofv3 kernel summary of ResNet-50. Each GPU step has its own time limit.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-rf}
for d in 18 50; do
  timeout -k 10 300 python bench_resnet.py --depth $d --batch_size 128 --steps 10 --warmup 3 \
    > gpurun_out/bench_resnet${d}_$TAG.log 2>&1 || { echo "bench r$d failed"; tail -30 gpurun_out/bench_resnet${d}_$TAG.log; exit 1; }
  tail -1 gpurun_out/bench_resnet${d}_$TAG.log
  timeout -k 10 300 python scripts/bench_torch_ref.py --model resnet$d --batch_size 128 --steps 10 --warmup 3 \
    > gpurun_out/torchref_r${d}_$TAG.log 2>&1 || { echo "torch ref r$d failed"; tail -20 gpurun_out/torchref_r${d}_$TAG.log; exit 1; }
  tail -1 gpurun_out/torchref_r${d}_$TAG.log
done
rm -rf gpurun_out/prof_r50_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_$TAG -o run -- python3 bench_resnet.py --depth 50 --batch_size 128 --steps 3 --warmup 1 \
  > gpurun_out/prof_r50_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_r50_$TAG.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof_r50_$TAG -name "*.db" | head -1) --min-calls 3 > gpurun_out/kernels_r50_$TAG.txt
head -40 gpurun_out/kernels_r50_$TAG.txt
