#!/bin/bash
# GPU parameter server tests + conv1-wgrad-tail A/B (one box session).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_r3_ps.sh || exit 1
bash scripts/gpu_r3_c1w.sh
