#!/bin/bash
# round-end style check: full GPU suite, smoke(), driver-style bench (N=1), long bench, forced-DP
# rehearsal of the 8-GPU default, ResNet-50/18 benches, MNIST kernel profile
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-fin}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" gpurun_out/pytest_gpu_$TAG.log | head; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke_$TAG.log; exit 1; }
grep "smoke ok" gpurun_out/smoke_$TAG.log
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b20_$TAG.log 2>&1 || { echo "bench failed"; cat gpurun_out/b20_$TAG.log; exit 1; }
  grep -o '"value": [0-9.]*.*"ms_per_step": [0-9.]*' gpurun_out/b20_$TAG.log
done
timeout -k 10 120 python bench.py --steps 1000 --warmup 100 > gpurun_out/blong_$TAG.log 2>&1 && grep -o '"value": [0-9.]*.*"ms_per_step": [0-9.]*' gpurun_out/blong_$TAG.log
timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --force_dp 1 --zero 1 > gpurun_out/bdp_$TAG.log 2>&1 && grep -o '"ms_per_step": [0-9.]*' gpurun_out/bdp_$TAG.log
timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 10 --warmup 3 > gpurun_out/rn50_$TAG.log 2>&1 && grep -o '"value": [0-9.]*.*"ms_per_step": [0-9.]*' gpurun_out/rn50_$TAG.log
timeout -k 10 300 python bench_resnet.py --depth 18 --batch_size 128 --steps 10 --warmup 3 > gpurun_out/rn18_$TAG.log 2>&1 && grep -o '"value": [0-9.]*.*"ms_per_step": [0-9.]*' gpurun_out/rn18_$TAG.log
rm -rf gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 200 --warmup 20 --phases 0 > gpurun_out/prof_$TAG.log 2>&1 && python scripts/prof_summary.py $(find gpurun_out/prof_$TAG -name "*.db" | head -1) --min-calls 100 > gpurun_out/kernels_$TAG.txt && cat gpurun_out/kernels_$TAG.txt
