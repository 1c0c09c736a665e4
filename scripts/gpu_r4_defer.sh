#!/bin/bash
# GradJoin deferral: ResNet GPU tests, interleaved ResNet-50 b128 A/B (TFD_JOIN_DEFER 0/1), kernel table
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_resnet_gpu.py > gpurun_out/r4_defer_tests.log 2>&1 \
  || { tail -30 gpurun_out/r4_defer_tests.log; exit 1; }
tail -1 gpurun_out/r4_defer_tests.log
for i in 1 2 3; do
  line="run $i"
  for d in 0 1; do
    r=$(TFD_JOIN_DEFER=$d timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || { echo "bench defer=$d failed"; exit 1; }
    line="$line | defer$d $r"
  done
  echo "$line" | tee -a gpurun_out/r4_defer_ab.log
done
rm -rf gpurun_out/prof_df
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_df -o run -- python3 bench_resnet.py --depth 50 --batch_size 128 --steps 10 --warmup 3 > gpurun_out/prof_df.log 2>&1 || { tail -20 gpurun_out/prof_df.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof_df -name "*.db" | head -1) > gpurun_out/rn50_kernels_defer.txt
rm -rf gpurun_out/prof_df
grep -E "bn_partial|bn_final" gpurun_out/rn50_kernels_defer.txt | cut -c1-100
