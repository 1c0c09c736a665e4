#!/bin/bash
# IPC DP-bench stress: 2 ranks on one GPU, repeated, per variant (env prefix); counts failures.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TFD_IPC_SPIN_MS=5000
port=29570
for variant in "${@}"; do
  fails=0
  for i in 1 2 3 4; do
    port=$((port+1))
    env $variant timeout -k 10 100 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --steps 20 --warmup 5 --min_warmup_ms 50 --phases 0 > gpurun_out/d_$port.log 2>&1 || fails=$((fails+1))
  done
  echo "[$variant] failures: $fails / 4"
done
