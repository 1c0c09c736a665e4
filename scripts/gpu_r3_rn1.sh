#!/bin/bash
# ResNet: BN-backward statistics in the dgrad epilogue -- tests, then an interleaved ResNet-50 b128 A/B
# (bench_resnet.py --bn_bwd_stats 1/0) and a kernel table of the new default.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py tests/test_conv_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rn1.log 2>&1 \
  || { echo "resnet tests failed"; tail -40 gpurun_out/pytest_rn1.log; exit 1; }
echo "resnet tests: $(tail -1 gpurun_out/pytest_rn1.log)"
for r in 1 2 3; do
  for arm in 1 0; do
    timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 --bn_bwd_stats $arm > gpurun_out/rn1.tmp 2>&1 \
      || { echo "bench failed"; tail -20 gpurun_out/rn1.tmp; exit 1; }
    echo "bn_bwd_stats=$arm $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rn1.tmp) $(grep -o '"value": [0-9.]*' gpurun_out/rn1.tmp)" | tee -a gpurun_out/ab_rn1.log
  done
done
rm -rf gpurun_out/prof_rn1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn1 -o run -- python3 bench_resnet.py --depth 50 --batch_size 128 --steps 10 --warmup 3 > gpurun_out/prof_rn1.log 2>&1 \
  || { echo "rocprof failed"; tail -20 gpurun_out/prof_rn1.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof_rn1 -name "*.db" | head -1) --min-calls 5 > gpurun_out/kernels_rn1.txt 2>&1
head -30 gpurun_out/kernels_rn1.txt
rm -rf gpurun_out/prof_rn1
