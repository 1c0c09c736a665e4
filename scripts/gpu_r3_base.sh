#!/bin/bash
# Round-3 baseline at HEAD: full GPU suite, 1-GPU bench, kernel table, PMC passes.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed: $?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python bench.py --steps 1000 --warmup 20 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; cat gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 200 --warmup 20 --phases 0 > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof -name "*.db" | head -1) > gpurun_out/kernels.txt 2>&1 || true
bash scripts/gpu_pmc.sh
