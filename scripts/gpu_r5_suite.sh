#!/bin/bash
# Round 5: the whole GPU suite, smoke, the driver-style MNIST bench twice, ResNet-50 b128.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=gpurun_out/r5_suite.log
: > $L
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_suite_pytest.log 2>&1 || { tail -40 gpurun_out/r5_suite_pytest.log; exit 1; }
tail -1 gpurun_out/r5_suite_pytest.log | tee -a $L
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 | tee -a $L
for r in 1 2; do
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/fb.tmp 2>&1 || { cat gpurun_out/fb.tmp; exit 1; }
  echo "driver-style 20/5: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fb.tmp) $(grep -o '"value": [0-9.]*' gpurun_out/fb.tmp)" | tee -a $L
done
timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/fb.tmp 2>&1 || { tail -20 gpurun_out/fb.tmp; exit 1; }
echo "resnet50 b128: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fb.tmp)" | tee -a $L
