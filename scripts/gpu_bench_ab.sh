#!/bin/bash
# Interleaved A/B/C/... of bench.py argument sets on one lease: ARGS_A, ARGS_B (and optional ARGS_C,
# ARGS_D), REPS rounds, at 20/5 and 1000/100 (SWEEPS="20 5;1000 100" overrides). ENV_A .. ENV_D:
# extra environment for that arm (e.g. ENV_B="TFD_NATIVE_LIB=$PWD/tensorflow_distributed_amd/_C_x.so").
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
IFS=';' read -ra SW <<< "${SWEEPS:-20 5;1000 100}"
for r in $(seq 1 ${REPS:-2}); do
  for v in A B C D; do
    eval "args=\${ARGS_$v-__unset__}"
    [ "$args" = "__unset__" ] && continue
    eval "envs=\${ENV_$v-}"
    for sw in "${SW[@]}"; do
      set -- $sw
      env $envs timeout -k 10 120 python bench.py --steps $1 --warmup $2 $args > gpurun_out/ab.log 2>&1 || { echo "bench failed"; cat gpurun_out/ab.log; exit 1; }
      echo "$v [$args${envs:+ $envs}] $1/$2: $(grep -o 'ms_per_step": [0-9.]*' gpurun_out/ab.log)"
    done
  done
done
