#!/bin/bash
# Round 5 heap bisection, call 3 (stub collective): no side stream at all; then the side stream with
# every hand-off issued from the main thread after backward(). Runs that may abort go last.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=gpurun_out/r5_heap3.log
: > $L
run() {
  local n=$1 t=$2; shift 2
  echo "== $n: $*" | tee -a $L
  MALLOC_CHECK_=3 MALLOC_PERTURB_=165 timeout -k 10 $t "$@" > gpurun_out/r5_heap3_$n.log 2>&1
  local rc=$?
  tail -12 gpurun_out/r5_heap3_$n.log | tee -a $L
  echo "rc=$rc" | tee -a $L
  return $rc
}
TFD_LOOP_NOSTREAM=1 run stub1_nostream 300 python -X faulthandler scripts/debug/rn_configure_loop.py stub1 60 &&
TFD_LOOP_DEFER=1 run stub1_defer 300 python -X faulthandler scripts/debug/rn_configure_loop.py stub1 60
