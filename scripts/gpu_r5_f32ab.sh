#!/bin/bash
# Round 5: fp32 step after a core change: fp32 numerics tests, then the kernel table and bench.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mnist_fp32_gpu.py > gpurun_out/r5_f32_t.log 2>&1 || { tail -30 gpurun_out/r5_f32_t.log; exit 1; }
tail -1 gpurun_out/r5_f32_t.log
bash scripts/gpu_r5_f32prof.sh
for i in 1 2; do timeout -k 10 120 python bench.py --dtype fp32 > gpurun_out/r5_f32_d$i.log 2>&1 || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_f32_d$i.log; done
