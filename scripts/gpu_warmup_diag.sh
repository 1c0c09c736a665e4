#!/bin/bash
# Short-run vs long-run bench gap diagnosis (one lease): per-replay event timeline, then the
# driver's 20/5 invocation three times and a 1000/100 run.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 180 python scripts/debug/warmup_ramp.py --steps 400 > gpurun_out/ramp.log 2>&1 || { echo "ramp failed"; tail -20 gpurun_out/ramp.log; exit 1; }
cat gpurun_out/ramp.log | grep -v amdgpu.ids
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/b20_$i.log 2>&1 || { echo "bench failed"; cat gpurun_out/b20_$i.log; exit 1; }
  grep ms/step gpurun_out/b20_$i.log
done
timeout -k 10 120 python bench.py --steps 1000 --warmup 100 > gpurun_out/b1000.log 2>&1 || { echo "bench failed"; cat gpurun_out/b1000.log; exit 1; }
grep ms/step gpurun_out/b1000.log
