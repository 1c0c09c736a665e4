#!/bin/bash
# Round 5: is the rccl1 capture/destroy heap failure ours (RcclComm user objects) or RCCL's?
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=gpurun_out/r5_rcclheap.log
: > $L
run() {
  echo "== $*" | tee -a $L
  MALLOC_CHECK_=3 MALLOC_PERTURB_=165 timeout -k 10 150 python -X faulthandler "$@" >> $L 2>&1
  echo "rc=$?" | tee -a $L
}
run scripts/debug/rccl_graph_loop.py ours 300
run scripts/debug/rccl_graph_loop.py torch 300
run scripts/debug/rn_configure_loop.py rccl1 40
run scripts/debug/rn_configure_loop.py rccl1 40
grep -c "ok" $L
