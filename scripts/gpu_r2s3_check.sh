#!/bin/bash
# conv/ResNet tests (new join test, 128-tile dgrad epilogue), ResNet-50 kernel profile, MNIST 20/5 bench with timed-region diagnostics
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv_ops_gpu.py tests/test_resnet_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_rn.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_rn.log; exit 1; }
tail -2 gpurun_out/pytest_rn.log
for i in 1 2 3; do
  TFD_BENCH_DIAG=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --phases 0 > gpurun_out/b20.log 2>&1 || { echo "bench failed"; cat gpurun_out/b20.log; exit 1; }
  grep -E "timed region|ms_per_step" gpurun_out/b20.log | sed 's/.*\("ms_per_step": [0-9.]*, "gpu_event_ms_per_step": [0-9.]*\).*/\1/'
done
rm -rf gpurun_out/prof_rn
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run -- python3 bench_resnet.py --depth 50 --batch_size 128 --steps 6 --warmup 2 > gpurun_out/prof_rn.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_rn.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof_rn -name "*.db" | head -1) --min-calls 6 > gpurun_out/kernels_rn.txt
head -30 gpurun_out/kernels_rn.txt
timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 10 --warmup 3 > gpurun_out/bench_rn50.log 2>&1 && grep -o '"value": [0-9.]*, "unit": "images/s".*"ms_per_step": [0-9.]*' gpurun_out/bench_rn50.log
timeout -k 10 300 python bench_resnet.py --depth 18 --batch_size 128 --steps 10 --warmup 3 > gpurun_out/bench_rn18.log 2>&1 && grep -o '"value": [0-9.]*, "unit": "images/s".*"ms_per_step": [0-9.]*' gpurun_out/bench_rn18.log
