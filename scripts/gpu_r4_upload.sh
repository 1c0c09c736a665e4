#!/bin/bash
# driver-style timed region with and without hipGraphUpload after capture (TFD_GRAPH_UPLOAD 0/1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2 3 4; do
  line="run $i"
  for up in 0 1; do
    r=$(TFD_GRAPH_UPLOAD=$up TFD_BENCH_DIAG=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 2>gpurun_out/up.err | grep -o '"ms_per_step": [0-9.]*\|"gpu_event_ms_per_step": [0-9.]*' | tr '\n' ' ') || { echo "bench up=$up failed"; tail -5 gpurun_out/up.err; exit 1; }
    d=$(grep -o "host launch [0-9.]* us, sync wait [0-9.]* us" gpurun_out/up.err | head -1)
    line="$line | up$up $r ($d)"
  done
  echo "$line" | tee -a gpurun_out/r4_upload.log
done
