#!/bin/bash
# IPC all-reduce microbenchmark at world 2 and 4 (ranks share the one GPU), event-timed and
# rocprofv3 kernel-traced. TAG names the outputs.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-ipc}
for w in 2 4; do
  for mb in 8 64; do
    timeout -k 10 120 python scripts/debug/ipc_bench.py --world $w --n 52096 --reps 200 --max_blocks $mb 2>&1 | grep '^{' | tee -a gpurun_out/ipc_$TAG.txt || exit 1
  done
done
rm -rf gpurun_out/prof_ipc_$TAG
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ipc_$TAG -o run -- python3 scripts/debug/ipc_bench.py --world 2 --n 52096 --reps 200 > gpurun_out/prof_ipc_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_ipc_$TAG.log; exit 1; }
for db in $(find gpurun_out/prof_ipc_$TAG -name "*.db"); do python scripts/prof_summary.py $db --min-calls 100; done | tee gpurun_out/ipc_kernels_$TAG.txt
