#!/bin/bash
# One-GPU step A/B: conv1-wgrad tail (conflict-free x pitch + prefetch), bf16 wgrad slabs, fc1-weight
# Adam deferred into the next fc1 forward; engine/DP/ResNet tests on the new code first (a test
# failure is reported, a crash or timeout ends the script).
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_mnist_engine_gpu.py tests/test_dropout_curve_gpu.py tests/test_dp_transport_gpu.py "tests/test_resnet_gpu.py::test_resnet_rccl_bucketed_world1_equals_no_comm" -q --timeout 120 --timeout-method thread > gpurun_out/pytest_c1w.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_c1w.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/pytest_c1w.log; exit 1; fi
ROUNDS=3 TAG=c1w ARMS="base|base|;old|c1wold|;xs|c1wxs|;wgbf|base|--wg2_bf16 1;defer|base|--defer_fc1_adam 1;dwg|base|--defer_fc1_adam 1 --wg2_bf16 1" bash scripts/gpu_ab3.sh || exit 1
TFD_NATIVE_LIB=$PWD/tensorflow_distributed_amd/_C.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dwg -o run -- python3 bench.py --steps 200 --warmup 20 --phases 0 --defer_fc1_adam 1 --wg2_bf16 1 > gpurun_out/prof_dwg.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_dwg.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/prof_dwg -name "*.db" | head -1) > gpurun_out/kernels_dwg.txt 2>&1; head -14 gpurun_out/kernels_dwg.txt; rm -rf gpurun_out/prof_dwg
