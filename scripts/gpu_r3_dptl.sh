#!/bin/bash
# kernel table + per-step timeline of the DP rehearsal (RCCL world 1, SFB + ZeRO-1 = the 8-GPU default)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for z in 1; do
rm -rf gpurun_out/prof_dp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dp -o run -- python3 bench.py --steps 200 --warmup 20 --phases 0 --force_dp 1 --zero $z > gpurun_out/prof_dp.log 2>&1 \
  || { echo "rocprof failed"; tail -20 gpurun_out/prof_dp.log; exit 1; }
db=$(find gpurun_out/prof_dp -name "*.db" | head -1)
python scripts/prof_summary.py $db > gpurun_out/kernels_dp.txt 2>&1
python scripts/prof_timeline.py $db > gpurun_out/timeline_dp.txt 2>&1
cat gpurun_out/kernels_dp.txt gpurun_out/timeline_dp.txt
rm -rf gpurun_out/prof_dp
done
