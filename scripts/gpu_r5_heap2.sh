#!/bin/bash
# Round 5 heap bisection, call 2: the ResNet DP capture cycle with the collective replaced by torch ops
# (stub1), then the IPC comm with the fp32 in-place wire. Runs that may abort go last.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=gpurun_out/r5_heap2.log
: > $L
run() {
  local n=$1 t=$2; shift 2
  echo "== $n: $*" | tee -a $L
  MALLOC_CHECK_=3 MALLOC_PERTURB_=165 timeout -k 10 $t "$@" > gpurun_out/r5_heap2_$n.log 2>&1
  local rc=$?
  tail -12 gpurun_out/r5_heap2_$n.log | tee -a $L
  echo "rc=$rc" | tee -a $L
  return $rc
}
run stub1_drop 300 python -X faulthandler scripts/debug/rn_configure_loop.py stub1 60 &&
TFD_LOOP_FP32=1 run ipc1_fp32_drop 300 python -X faulthandler scripts/debug/rn_configure_loop.py ipc1 60
