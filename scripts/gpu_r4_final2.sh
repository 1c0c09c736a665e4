#!/bin/bash
# End-of-session check: full GPU suite, smoke, driver-style and long benches, the DP rehearsal of
# the 8-GPU default, ResNet-50, and a kernel table + timeline of the one-GPU step.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=gpurun_out/final_r4s2.log
: > $L
:
:
:
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 | tee -a $L
for r in 1 2 3; do
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/fb.tmp 2>&1 || { cat gpurun_out/fb.tmp; exit 1; }
  echo "driver-style 20/5: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fb.tmp) $(grep -o '"value": [0-9.]*' gpurun_out/fb.tmp)" | tee -a $L
done
tail -1 gpurun_out/fb.tmp > gpurun_out/bench_final_r4s2.json
timeout -k 10 180 python bench.py --steps 1000 --warmup 20 > gpurun_out/fb.tmp 2>&1 || { cat gpurun_out/fb.tmp; exit 1; }
echo "1000 steps: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fb.tmp)" | tee -a $L
timeout -k 10 180 python bench.py --steps 1000 --warmup 20 --force_dp 1 --zero 1 > gpurun_out/fb.tmp 2>&1 || { cat gpurun_out/fb.tmp; exit 1; }
echo "DP rehearsal (rccl world 1, sfb + zero): $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fb.tmp)" | tee -a $L
timeout -k 10 180 python bench.py --steps 1000 --warmup 20 --force_dp 1 --zero 0 > gpurun_out/fb.tmp 2>&1 || { cat gpurun_out/fb.tmp; exit 1; }
echo "DP rehearsal (rccl world 1, sfb): $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fb.tmp)" | tee -a $L
for r in 1 2; do
  timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/fb.tmp 2>&1 || { tail -20 gpurun_out/fb.tmp; exit 1; }
  echo "resnet50 b128: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fb.tmp) $(grep -o '"value": [0-9.]*' gpurun_out/fb.tmp)" | tee -a $L
done
SUITE=0 bash scripts/gpu_r3_tl.sh > gpurun_out/tl_final.txt 2>&1; cat gpurun_out/tl_final.txt | tail -22
timeout -k 10 240 python bench_resnet.py --depth 18 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/fb.tmp 2>&1 || { tail -20 gpurun_out/fb.tmp; exit 1; }
echo "resnet18 b128: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fb.tmp) $(grep -o '"value": [0-9.]*' gpurun_out/fb.tmp)" | tee -a $L
rm -rf gpurun_out/prof_rn50_final
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn50_final -o run -- python bench_resnet.py --depth 50 --batch_size 128 --steps 15 --warmup 3 > gpurun_out/prof_rn50_final.log 2>&1 || { tail -20 gpurun_out/prof_rn50_final.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof_rn50_final -name "*.db" | head -1) > gpurun_out/resnet50_kernels_final_r4s2.txt && echo "resnet50 kernel table written" | tee -a $L
