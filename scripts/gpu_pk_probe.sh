#!/bin/bash
# Packed-fp32 VALU probe: determinism of the pk variant (_C_pk.so) with 1 process vs 4 processes
# sharing the GPU (VALU conv1 path and fused conv12 path), and its bench time vs the default build.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PK=$PWD/tensorflow_distributed_amd/_C_pk.so
for cfg in "1 1" "4 1" "4 0"; do
  set -- $cfg
  echo "== pk world $1 unfused $2"
  TFD_NATIVE_LIB=$PK timeout -k 10 300 python scripts/debug/determinism.py $1 $2 > gpurun_out/pk_det_$1_$2.log 2>&1 || { echo "determinism failed"; tail -20 gpurun_out/pk_det_$1_$2.log; exit 1; }
  grep "max diff\|vs rank0" gpurun_out/pk_det_$1_$2.log | cut -c1-400
done
echo "== base world 4 unfused 1"
timeout -k 10 300 python scripts/debug/determinism.py 4 1 > gpurun_out/base_det.log 2>&1 || { echo "determinism failed"; tail -20 gpurun_out/base_det.log; exit 1; }
grep "max diff\|vs rank0" gpurun_out/base_det.log | cut -c1-400
for r in 1 2; do
  for lib in base pk; do
    L=$PWD/tensorflow_distributed_amd/_C.so; [ $lib = pk ] && L=$PK
    TFD_NATIVE_LIB=$L timeout -k 10 120 python bench.py --steps 1000 --warmup 100 > gpurun_out/pkb.log 2>&1 || { echo "bench failed"; tail gpurun_out/pkb.log; exit 1; }
    echo "$lib: $(grep -o 'ms_per_step": [0-9.]*' gpurun_out/pkb.log)"
  done
done
