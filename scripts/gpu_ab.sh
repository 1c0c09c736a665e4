#!/bin/bash
# Engine GPU tests, then interleaved 1-GPU bench A/B of engine switches (same box, same process
# order each round). ARGS_A / ARGS_B: extra bench.py flags of the two arms.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-ab}
TESTS=${TESTS:-tests/test_mnist_engine_gpu.py tests/test_ipc_gpu.py}
timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
for r in 1 2 3; do
  for arm in A B; do
    if [ $arm = A ]; then X="$ARGS_A"; else X="$ARGS_B"; fi
    timeout -k 10 120 python bench.py --steps 2000 --warmup 200 $X > gpurun_out/ab_$TAG.tmp 2>&1 \
      || { echo "bench $arm failed"; cat gpurun_out/ab_$TAG.tmp; exit 1; }
    echo "$arm [$X] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$TAG.tmp)" | tee -a gpurun_out/ab_$TAG.log
  done
done
