#!/bin/bash
# whole-step bit-reproducibility (scripts/debug/step_det.py) for the default build and variants
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for l in base noglds c1wv; do
  if [ $l = base ]; then lib=$PWD/tensorflow_distributed_amd/_C.so; else lib=$PWD/tensorflow_distributed_amd/_C_$l.so; fi
  echo "== $l" | tee -a gpurun_out/sdet.log
  TFD_NATIVE_LIB=$lib timeout -k 10 200 python -u scripts/debug/step_det.py 60 5 2>&1 | grep -v Warn | tee -a gpurun_out/sdet.log
done
