#!/bin/bash
# A/B several native-library variants (tensorflow_distributed_amd/_C_<name>.so) on one GPU box:
# bench + rocprofv3 kernel summary for each. VARIANTS="base bk128 ..." ("base" = _C.so).
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
for v in ${VARIANTS:-base}; do
  if [ "$v" = "base" ]; then lib=tensorflow_distributed_amd/_C.so; else lib=tensorflow_distributed_amd/_C_$v.so; fi
  export TFD_NATIVE_LIB=$PWD/$lib
  timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$v.log 2>&1 || { echo "bench $v failed"; cat gpurun_out/bench_$v.log; exit 1; }
  echo "== $v: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_$v.log)"
  rm -rf gpurun_out/prof_$v
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$v -o run -- python3 bench.py --steps 200 --warmup 20 ${BENCH_ARGS:-} > gpurun_out/prof_$v.log 2>&1 || { echo "rocprof $v failed"; tail -30 gpurun_out/prof_$v.log; exit 1; }
  python scripts/prof_summary.py $(find gpurun_out/prof_$v -name "*.db" | head -1) > gpurun_out/kernels_$v.txt
  cat gpurun_out/kernels_$v.txt
done
