#!/bin/bash
# Round 5: host-heap corruption after destroying captured two-stream DP graphs.
# Runs that may abort go last; every step under its own time limit, chained with &&.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=gpurun_out/r5_heap.log
: > $L
run() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  echo "== $n: $*" | tee -a $L
  MALLOC_CHECK_=3 MALLOC_PERTURB_=165 timeout -k 10 $t "$@" > gpurun_out/r5_heap_$n.log 2>&1
  local rc=$?
  tail -5 gpurun_out/r5_heap_$n.log | tee -a $L
  echo "rc=$rc" | tee -a $L
  return $rc
}
run twin_pooled_drop 240 python -X faulthandler scripts/debug/heap_twin.py pooled 60 drop &&
run twin_fresh_drop 240 python -X faulthandler scripts/debug/heap_twin.py fresh 60 drop &&
run rn_none_drop 300 python -X faulthandler scripts/debug/rn_configure_loop.py none 30 &&
run rn_ipc1_keep 300 python -X faulthandler scripts/debug/rn_configure_loop.py ipc1 40 -1 1 keep &&
run rn_ipc1_drop 300 python -X faulthandler scripts/debug/rn_configure_loop.py ipc1 60
