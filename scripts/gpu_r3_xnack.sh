#!/bin/bash
# code objects built for gfx950:xnack- (XNACK off, as on this pool) vs the default xnack-any build
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/tensorflow_distributed_amd
TEST_LIBS="xnm" ROUNDS=3 TAG=xnm PROF=0 ARMS="xnm|xnm|;base|base|" bash scripts/gpu_ab3.sh || exit 1
for r in 1 2 3; do
  for arm in xnm base; do
    if [ $arm = base ]; then lib=$L/_C.so; else lib=$L/_C_$arm.so; fi
    TFD_NATIVE_LIB=$lib timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/xnm.tmp 2>&1 \
      || { echo "bench failed"; tail -20 gpurun_out/xnm.tmp; exit 1; }
    echo "resnet50 $arm $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/xnm.tmp)" | tee -a gpurun_out/ab_xnm.log
  done
done
