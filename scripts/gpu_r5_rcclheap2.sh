#!/bin/bash
# Round 5: RCCL capture/destroy cycles with the ResNet backward on the caller's thread (10 x 40
# cycles under glibc heap checks), then the ResNet GPU tests and a ResNet-50 bench line.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=gpurun_out/r5_rcclheap2.log
: > $L
fails=0
for i in 1 2 3 4 5 6 7 8 9 10; do
  MALLOC_CHECK_=3 MALLOC_PERTURB_=165 timeout -k 10 150 python -X faulthandler scripts/debug/rn_configure_loop.py rccl1 40 >> $L 2>&1
  rc=$?
  echo "run $i rc=$rc" | tee -a $L
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
  [ $rc -ne 0 ] && fails=$((fails+1))
done
echo "failed runs: $fails / 10" | tee -a $L
timeout -k 10 900 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_rn_t.log 2>&1 || { tail -30 gpurun_out/r5_rn_t.log; exit 1; }
tail -1 gpurun_out/r5_rn_t.log
timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/r5_rn_b.log 2>&1 || { tail -20 gpurun_out/r5_rn_b.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_rn_b.log
