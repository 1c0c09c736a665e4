#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=$PWD/tensorflow_distributed_amd
for v in base px1 g2048 g4096 g4096p1; do
  if [ $v = base ]; then lib=$L/_C.so; else lib=$L/_C_$v.so; fi
  echo -n "$v: "; TFD_NATIVE_LIB=$lib timeout -k 10 120 python tools/debug/pool_probe.py || exit 1
  echo -n "$v rows: "; TFD_NATIVE_LIB=$lib timeout -k 10 120 python tools/debug/pool_probe.py rows || exit 1
done
