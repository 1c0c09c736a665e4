#!/bin/bash
# where does the bench's state diverge between runs of the same binary? (TFD_BENCH_DIAG digests)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2 3 4 5 6; do
  TFD_BENCH_DIAG=1 timeout -k 10 120 python bench.py --steps 200 --warmup 20 --min_warmup_ms 0 --phases 0 > gpurun_out/det2.tmp 2>&1 || { cat gpurun_out/det2.tmp; exit 1; }
  echo "run $r" | tee -a gpurun_out/det2.log
  grep -E "# digest|# world" gpurun_out/det2.tmp | tee -a gpurun_out/det2.log
done
