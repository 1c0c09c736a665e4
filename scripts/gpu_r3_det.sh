#!/bin/bash
# Is the bench's final loss a deterministic function of the run? Same binary, varied untimed warm-up.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for mw in 0 0 300 300 600 0; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --min_warmup_ms $mw > gpurun_out/det.tmp 2>&1 || { cat gpurun_out/det.tmp; exit 1; }
  echo "min_warmup_ms=$mw $(grep -o '# world.*' gpurun_out/det.tmp)" | tee -a gpurun_out/det.log
done
for ph in 0 0; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --min_warmup_ms 0 --phases $ph > gpurun_out/det.tmp 2>&1 || { cat gpurun_out/det.tmp; exit 1; }
  echo "phases=$ph $(grep -o '# world.*' gpurun_out/det.tmp)" | tee -a gpurun_out/det.log
done
timeout -k 10 200 python scripts/debug/determinism.py 1 0 > gpurun_out/det_repeat.log 2>&1 || { tail -20 gpurun_out/det_repeat.log; exit 1; }
tail -5 gpurun_out/det_repeat.log
