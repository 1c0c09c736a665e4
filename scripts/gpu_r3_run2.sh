set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=state ARMS="base100|base|--data strokes --state_steps 100;skip100|skip0|--data strokes --state_steps 100;rnd0|base|--data random --state_steps 0;skiprnd0|skip0|--data random --state_steps 0" bash scripts/gpu_ab3.sh || exit 1
timeout -k 10 900 python -u -m pytest tests/test_ipc_gpu.py tests/test_mnist_engine_gpu.py tests/test_dp_transport_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r3b.log 2>&1; echo "pytest rc=$?"; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_r3b.log | tail -70; grep -B2 -A25 "^E  " gpurun_out/pytest_r3b.log | head -120
