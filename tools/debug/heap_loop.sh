set -o pipefail
mkdir -p gpurun_out/r6q
export MALLOC_CHECK_=3 MALLOC_PERTURB_=165 HSA_ENABLE_IPC_MODE_LEGACY=0
for m in ipc1 ipc1 stub1 rccl1; do
  echo "== $m $(date +%T)"
  timeout -k 10 200 python -u tools/debug/rn_configure_loop.py $m 100 >> gpurun_out/r6q/loop_$m.log 2>&1
  echo "rc $?"
done
