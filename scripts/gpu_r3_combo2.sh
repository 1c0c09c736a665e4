#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash scripts/gpu_r3_c1w.sh || exit 1
timeout -k 10 200 python -u scripts/debug/ps_probe.py > gpurun_out/ps_probe.log 2>&1; echo "probe rc=$?"; tail -5 gpurun_out/ps_probe.log
