#!/bin/bash
# Interleaved A/B over arms "name|lib|bench args" (';'-separated in ARMS; lib "base" = _C.so, else
# _C_<lib>.so), ROUNDS rounds of bench.py; optional engine tests per lib (TEST_LIBS) and a rocprofv3
# kernel table of the first arm (PROF=1). Large profiler databases are deleted after summarising
# (gpurun copies back at most 64 MiB of gpurun_out/).
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-ab3}
STEPS=${STEPS:-1000}
lib() { if [ "$1" = "base" ]; then echo $PWD/tensorflow_distributed_amd/_C.so; else echo $PWD/tensorflow_distributed_amd/_C_$1.so; fi; }
for l in ${TEST_LIBS:-}; do
  TFD_NATIVE_LIB=$(lib $l) timeout -k 10 300 python -u -m pytest ${TEST_FILES:-tests/test_mnist_engine_gpu.py} -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_${TAG}_$l.log 2>&1 || { echo "pytest $l failed"; tail -30 gpurun_out/pytest_${TAG}_$l.log; exit 1; }
  echo "tests $l: $(tail -1 gpurun_out/pytest_${TAG}_$l.log)"
done
IFS=';' read -ra AR <<< "$ARMS"
for r in $(seq 1 ${ROUNDS:-3}); do
  for arm in "${AR[@]}"; do
    IFS='|' read -r name l args <<< "$arm"
    TFD_NATIVE_LIB=$(lib $l) timeout -k 10 180 python bench.py --steps $STEPS --warmup 20 $args > gpurun_out/ab_$TAG.tmp 2>&1 \
      || { echo "bench $name failed"; cat gpurun_out/ab_$TAG.tmp; exit 1; }
    echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$TAG.tmp) $(grep -o '# world.*' gpurun_out/ab_$TAG.tmp)" | tee -a gpurun_out/ab_$TAG.log
  done
done
if [ "${PROF:-0}" = "1" ]; then
  IFS='|' read -r name l args <<< "${AR[0]}"
  rm -rf gpurun_out/prof_$TAG
  TFD_NATIVE_LIB=$(lib $l) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 200 --warmup 20 --phases 0 $args > gpurun_out/prof_$TAG.log 2>&1 \
    || { echo "rocprof failed"; tail -30 gpurun_out/prof_$TAG.log; exit 1; }
  python scripts/prof_summary.py $(find gpurun_out/prof_$TAG -name "*.db" | head -1) > gpurun_out/kernels_$TAG.txt 2>&1
  cat gpurun_out/kernels_$TAG.txt
  rm -rf gpurun_out/prof_$TAG
fi
