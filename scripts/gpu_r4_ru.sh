#!/bin/bash
# rows per batch of the BN passes (TFD_BN_RU) 4 (base) / 2 / 8, ResNet-50 b128 interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/tensorflow_distributed_amd
for i in 1 2 3; do
  line="run $i"
  for arm in base ru2 ru8; do
    if [ $arm = base ]; then lib=$L/_C.so; else lib=$L/_C_$arm.so; fi
    r=$(TFD_NATIVE_LIB=$lib timeout -k 10 240 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || { echo "bench $arm failed"; exit 1; }
    line="$line | $arm $r"
  done
  echo "$line" | tee -a gpurun_out/r4_ru_ab.log
done
