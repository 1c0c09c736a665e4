#!/bin/bash
# Round 5 heap bisection, call 4: ready events recorded inside backward, side-stream work issued from
# the main thread (stub collective, then the real IPC comm).
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=gpurun_out/r5_heap4.log
: > $L
run() {
  local n=$1 t=$2; shift 2
  echo "== $n: $*" | tee -a $L
  MALLOC_CHECK_=3 MALLOC_PERTURB_=165 timeout -k 10 $t "$@" > gpurun_out/r5_heap4_$n.log 2>&1
  local rc=$?
  tail -12 gpurun_out/r5_heap4_$n.log | tee -a $L
  echo "rc=$rc" | tee -a $L
  return $rc
}
TFD_LOOP_SPLIT=1 run stub1_split 300 python -X faulthandler scripts/debug/rn_configure_loop.py stub1 80 &&
TFD_LOOP_SPLIT=1 run ipc1_split 300 python -X faulthandler scripts/debug/rn_configure_loop.py ipc1 80
