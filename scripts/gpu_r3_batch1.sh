#!/bin/bash
# batch: PMC + wgrad A/B, then the ResNet side-finalize A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_r3_pmc_ab2.sh && bash scripts/gpu_r3_rn2.sh
