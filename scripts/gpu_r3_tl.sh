#!/bin/bash
# Full GPU suite at HEAD + rocprofv3 kernel trace of the one-GPU bench with a per-step timeline.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ "${SUITE:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1 \
    || { echo "gpu suite failed"; tail -30 gpurun_out/pytest_gpu_full.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu_full.log
fi
rm -rf gpurun_out/prof_tl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tl -o run -- python3 bench.py --steps 200 --warmup 20 --phases 0 ${BENCH_ARGS:-} > gpurun_out/prof_tl.log 2>&1 \
  || { echo "rocprof failed"; tail -30 gpurun_out/prof_tl.log; exit 1; }
db=$(find gpurun_out/prof_tl -name "*.db" | head -1)
python scripts/prof_summary.py $db > gpurun_out/kernels_tl.txt 2>&1
python scripts/prof_timeline.py $db > gpurun_out/timeline_tl.txt 2>&1
cat gpurun_out/kernels_tl.txt gpurun_out/timeline_tl.txt
rm -rf gpurun_out/prof_tl
