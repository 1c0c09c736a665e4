#!/bin/bash
# Per-kernel rocprofv3 times of native-library variants (VARIANTS="base e1 ..."; _C_<name>.so).
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
lib() { if [ "$1" = "base" ]; then echo $PWD/tensorflow_distributed_amd/_C.so; else echo $PWD/tensorflow_distributed_amd/_C_$1.so; fi; }
for v in ${VARIANTS:-base}; do
  rm -rf gpurun_out/vprof_$v
  TFD_NATIVE_LIB=$(lib $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/vprof_$v -o run -- python3 bench.py --steps 200 --warmup 20 --phases 0 > gpurun_out/vprof_$v.log 2>&1 || { echo "prof $v failed"; tail -5 gpurun_out/vprof_$v.log; exit 1; }
  echo "== $v"; python scripts/prof_summary.py $(find gpurun_out/vprof_$v -name "*.db" | head -1) --min-calls 100 | grep -v "^kernel"
done
