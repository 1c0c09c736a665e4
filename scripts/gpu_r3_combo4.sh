#!/bin/bash
# conv2 wgrad bank-class pixel order (A/B vs natural order), conv1 x pitch 52 (A/B), engine oracle tests.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mnist_engine_gpu.py tests/test_dropout_curve_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_perm.log 2>&1; rc=$?
echo "engine tests rc=$rc"; tail -3 gpurun_out/pytest_perm.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
ROUNDS=3 TAG=perm ARMS="base|base|;noperm|noperm|;xs52|xs52|" PROF=1 bash scripts/gpu_ab3.sh
