#!/bin/bash
# per-kernel medians of timing-diagnosis builds (fc1_bwd without dX / without dW blocks; conv2_bwd
# without wgrad / without dgrad blocks) next to the base build.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for l in base fd1 fd2 cd1 cd2; do
  if [ "$l" = "base" ]; then lib=$PWD/tensorflow_distributed_amd/_C.so; else lib=$PWD/tensorflow_distributed_amd/_C_$l.so; fi
  rm -rf gpurun_out/prof_d
  TFD_NATIVE_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_d -o run -- python3 bench.py --steps 200 --warmup 20 --phases 0 --state_steps 0 > gpurun_out/prof_d.log 2>&1 \
    || { echo "rocprof $l failed"; tail -20 gpurun_out/prof_d.log; exit 1; }
  echo "== $l"; python scripts/prof_summary.py $(find gpurun_out/prof_d -name "*.db" | head -1) | head -8 | tee -a gpurun_out/diag.txt
  rm -rf gpurun_out/prof_d
done
