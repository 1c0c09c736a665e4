#!/bin/bash
# ResNet: BN-backward statistics also in the strided (phase) dgrads -- tests, ResNet-50 b128 A/B.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py tests/test_conv_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rn3.log 2>&1 \
  || { echo "resnet tests failed"; tail -40 gpurun_out/pytest_rn3.log; exit 1; }
echo "resnet tests: $(tail -1 gpurun_out/pytest_rn3.log)"
for r in 1 2 3; do
  for arm in 1 0; do
    TFD_BN_STATS_STRIDED=$arm timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/rn3.tmp 2>&1 \
      || { echo "bench failed"; tail -20 gpurun_out/rn3.tmp; exit 1; }
    echo "strided=$arm $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rn3.tmp)" | tee -a gpurun_out/ab_rn3.log
  done
done
