#!/bin/bash
# forward-apply inline finalize: LDS two-stage (in-tree) vs every thread from global (_C_fd.so), ResNet-50 b128
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/tensorflow_distributed_amd
for i in 1 2 3; do
  line="run $i"
  for arm in base fd; do
    if [ $arm = base ]; then lib=$L/_C.so; else lib=$L/_C_$arm.so; fi
    r=$(TFD_NATIVE_LIB=$lib timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || { echo "bench $arm failed"; exit 1; }
    line="$line | $arm $r"
  done
  echo "$line" | tee -a gpurun_out/r4_fd_ab.log
done
