set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for ov in 0 1 0 1; do timeout -k 10 200 python bench.py --steps 1000 --opt_overlap $ov > gpurun_out/b_ov$ov.log 2>&1 || exit 1; echo "ov=$ov $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_ov$ov.log)"; done
