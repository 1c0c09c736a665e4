#!/bin/bash
# Last check of the round-4 tree: GPU suite, smoke, driver-style bench, ResNet-50, then the MNIST
# fc-region Adam launch-shape A/B (scripts/gpu_r4_adam.sh) if the variant libraries are present.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=gpurun_out/last_r4.log
: > $L
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_last_r4.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_last_r4.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_last_r4.log | tee -a $L
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 | tee -a $L
for r in 1 2; do
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/fb.tmp 2>&1 || { cat gpurun_out/fb.tmp; exit 1; }
  echo "driver-style 20/5: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fb.tmp) $(grep -o '"value": [0-9.]*' gpurun_out/fb.tmp)" | tee -a $L
done
timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/fb.tmp 2>&1 || { tail -20 gpurun_out/fb.tmp; exit 1; }
echo "resnet50 b128: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fb.tmp) $(grep -o '"value": [0-9.]*' gpurun_out/fb.tmp)" | tee -a $L
if [ -f tensorflow_distributed_amd/_C_ad3200.so ]; then bash scripts/gpu_r4_adam.sh; fi
