#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 120 python scripts/debug/gemm256_probe.py > gpurun_out/g256.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/g256.log; exit $rc
