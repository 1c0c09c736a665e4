#!/bin/bash
# fc-region Adam launch shape: 1024 blocks x 2 strides (in-tree) vs 3200 x 1 / 1600 x 1, MNIST step (1000 steps) interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/tensorflow_distributed_amd
for i in 1 2 3; do
  line="run $i"
  for arm in base ad3200 ad1600u1; do
    if [ $arm = base ]; then lib=$L/_C.so; else lib=$L/_C_$arm.so; fi
    r=$(TFD_NATIVE_LIB=$lib timeout -k 10 120 python bench.py --steps 1000 --warmup 20 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || { echo "bench $arm failed"; exit 1; }
    line="$line | $arm $r"
  done
  echo "$line" | tee -a gpurun_out/r4_adam_ab.log
done
