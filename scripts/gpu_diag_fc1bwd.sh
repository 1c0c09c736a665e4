#!/bin/bash
# rocprofv3 kernel summaries of native-library variants (VARIANTS="base d1 d2 ..."; "base" = _C.so),
# e.g. the TFD_DIAG_FC1BWD timing-diagnosis builds that drop one part of fc1_bwd.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in ${VARIANTS:-d1 d2}; do
  if [ "$v" = "base" ]; then lib=$PWD/tensorflow_distributed_amd/_C.so; else lib=$PWD/tensorflow_distributed_amd/_C_$v.so; fi
  rm -rf gpurun_out/prof_$v
  TFD_NATIVE_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$v -o run -- python3 bench.py --steps 200 --warmup 20 > gpurun_out/prof_$v.log 2>&1 || { echo "prof $v failed"; tail -20 gpurun_out/prof_$v.log; exit 1; }
  python scripts/prof_summary.py $(find gpurun_out/prof_$v -name "*.db" | head -1) > gpurun_out/kernels_$v.txt
  echo "== $v"; grep -E "${GREP:-fc1_bwd|sum of}" gpurun_out/kernels_$v.txt
done
