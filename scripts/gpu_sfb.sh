#!/bin/bash
# SFB (sufficient-factor fc gradients) GPU check: DP transport + IPC engine tests, then forced-DP
# world-1 and 2-ranks-on-one-GPU benches with and without SFB.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-sfb}
timeout -k 10 600 python -u -m pytest tests/test_dp_transport_gpu.py tests/test_ipc_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error" gpurun_out/pytest_$TAG.log | tail -30; tail -50 gpurun_out/pytest_$TAG.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_$TAG.log | tail -40
for sfb in 0 1; do
  timeout -k 10 120 python bench.py --steps 500 --warmup 50 --force_dp 1 --fc_sfb $sfb > gpurun_out/bench_fdp_sfb$sfb.log 2>&1 || { echo "bench failed"; tail gpurun_out/bench_fdp_sfb$sfb.log; exit 1; }
  echo "force_dp sfb=$sfb: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_fdp_sfb$sfb.log) $(grep -o '"phases_ms": {[^}]*}' gpurun_out/bench_fdp_sfb$sfb.log)"
done
for sfb in 0 1; do
  timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 500 --warmup 50 --fc_sfb $sfb > gpurun_out/bench_dp2_sfb$sfb.log 2>&1 || { echo "bench dp2 failed"; tail gpurun_out/bench_dp2_sfb$sfb.log; exit 1; }
  echo "dp2 one GPU sfb=$sfb: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_dp2_sfb$sfb.log) $(grep -o '"phases_ms": {[^}]*}' gpurun_out/bench_dp2_sfb$sfb.log)"
done
