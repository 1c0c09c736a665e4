#!/bin/bash
# Round-4 first contact: 1-GPU bench, self-launched 2-rank bench with schedule probes, ResNet-50.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_base_b1.log 2>&1 && tail -2 gpurun_out/r4_base_b1.log &&
timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 20 > gpurun_out/r4_base_b2.log 2>&1 && grep -v "^\[W\|Gloo" gpurun_out/r4_base_b2.log | tail -8 &&
timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/r4_base_rn50.log 2>&1 && tail -2 gpurun_out/r4_base_rn50.log &&
timeout -k 10 300 python bench_resnet.py --gpus 2 --depth 18 --batch_size 32 --image 112 --steps 5 --warmup 2 > gpurun_out/r4_base_rn18x2.log 2>&1 && grep -v "^\[W\|Gloo" gpurun_out/r4_base_rn18x2.log | tail -8
