#!/bin/bash
# Interleaved ResNet bench of the in-tree build against every build_ab/<variant>.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2 3; do
  line="run $i head $(timeout -k 10 240 python bench_resnet.py --depth ${DEPTH:-50} --batch_size 128 --steps 20 --warmup 5 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" || { echo "head bench failed"; exit 1; }
  for d in build_ab/*/; do
    v=$(basename "$d")
    r=$(cd "$d" && timeout -k 10 240 python bench_resnet.py --depth ${DEPTH:-50} --batch_size 128 --steps 20 --warmup 5 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || { echo "$v bench failed"; exit 1; }
    line="$line | $v $r"
  done
  echo "$line" | tee -a gpurun_out/r4_rn_variants.log
done
