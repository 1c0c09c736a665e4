#!/bin/bash
# half-channel conv2 dgrad blocks (two blocks per CU in the one-launch conv2 backward): engine tests
# on that build, interleaved A/B, kernel table; then the timing-diagnosis tables.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TEST_LIBS="c2dh" TEST_FILES="tests/test_mnist_engine_gpu.py tests/test_dropout_curve_gpu.py" ROUNDS=3 TAG=c2dh ARMS="base|base|;c2dh|c2dh|" PROF=0 bash scripts/gpu_ab3.sh || exit 1
rm -rf gpurun_out/prof_h
TFD_NATIVE_LIB=$PWD/tensorflow_distributed_amd/_C_c2dh.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_h -o run -- python3 bench.py --steps 200 --warmup 20 --phases 0 --state_steps 0 > gpurun_out/prof_h.log 2>&1 \
  || { echo "rocprof failed"; tail -20 gpurun_out/prof_h.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof_h -name "*.db" | head -1) | head -9 | tee gpurun_out/kernels_c2dh.txt
rm -rf gpurun_out/prof_h
bash scripts/gpu_r3_diag.sh
