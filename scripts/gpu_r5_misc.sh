#!/bin/bash
# Round 5: topology (RCCL markers) + fp32 + engine tests, then the fp32 step's kernel table.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_graph_topology_gpu.py tests/test_mnist_fp32_gpu.py tests/test_mnist_engine_gpu.py > gpurun_out/r5_misc_t.log 2>&1 || { tail -40 gpurun_out/r5_misc_t.log; exit 1; }
tail -1 gpurun_out/r5_misc_t.log
bash scripts/gpu_r5_f32prof.sh
for i in 1 2; do timeout -k 10 120 python bench.py --dtype fp32 > gpurun_out/r5_misc_b.log 2>&1 || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_misc_b.log; done
