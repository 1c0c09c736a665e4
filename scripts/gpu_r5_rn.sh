#!/bin/bash
# Round 5: ResNet tests (magnitude oracle bounds, comm lifetime, capture/destroy cycles), the DP transport
# suite (dist_main schedule probes, ResNet Supervisor services), a one-GPU ResNet-50 bench line.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_resnet_gpu.py tests/test_dp_transport_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5_rn_pytest.log 2>&1 || { tail -60 gpurun_out/r5_rn_pytest.log; exit 1; }
tail -3 gpurun_out/r5_rn_pytest.log
timeout -k 10 300 python bench_resnet.py --depth 50 --batch_size 128 --steps 20 --warmup 5 > gpurun_out/r5_rn_bench.log 2>&1 || { tail -20 gpurun_out/r5_rn_bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_rn_bench.log
