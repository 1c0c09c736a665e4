#!/bin/bash
# Round-4 check: graph-topology + engine + DP bench tests, 1-GPU bench, self-launched probes at 2 ranks.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TESTS:-"tests/test_graph_topology_gpu.py tests/test_mnist_engine_gpu.py"}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r4_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "PASS|FAIL|Error" gpurun_out/r4_tests.log | tail -30; tail -40 gpurun_out/r4_tests.log; exit 1; }
grep -cE "PASSED" gpurun_out/r4_tests.log; tail -1 gpurun_out/r4_tests.log
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_b1.log 2>&1 && tail -2 gpurun_out/r4_b1.log | cut -c1-400 &&
timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 20 > gpurun_out/r4_b2.log 2>&1 && grep -v "^\[W\|Gloo" gpurun_out/r4_b2.log | tail -6 | cut -c1-600
