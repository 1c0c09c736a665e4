#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python scripts/debug/resnet_oracle_rel.py > gpurun_out/r5_resnet_oracle_rel.log 2>&1 || { tail -20 gpurun_out/r5_resnet_oracle_rel.log; exit 1; }
cat gpurun_out/r5_resnet_oracle_rel.log
