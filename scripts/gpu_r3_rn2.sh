#!/bin/bash
# ResNet: side-stream BN-backward finalize -- tests, interleaved ResNet-50 b128 A/B (--bn_final_side 1/0).
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rn2.log 2>&1 \
  || { echo "resnet tests failed"; tail -40 gpurun_out/pytest_rn2.log; exit 1; }
echo "resnet tests: $(tail -1 gpurun_out/pytest_rn2.log)"
for r in 1 2 3; do
  for arm in 1 0; do
    timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 --bn_final_side $arm > gpurun_out/rn2.tmp 2>&1 \
      || { echo "bench failed"; tail -20 gpurun_out/rn2.tmp; exit 1; }
    echo "bn_final_side=$arm $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rn2.tmp) $(grep -o '"value": [0-9.]*' gpurun_out/rn2.tmp)" | tee -a gpurun_out/ab_rn2.log
  done
done
