#!/bin/bash
# PMC counter passes (kernel-trace only, no sys/runtime trace) over a short bench run.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
# PMC_SETS="A B C;D E" overrides the default passes (';' separates passes)
DEFAULT_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE;SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM;SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC TCC_HIT_sum TCC_MISS_sum;FETCH_SIZE;WRITE_SIZE"
IFS=';' read -ra SETS <<< "${PMC_SETS:-$DEFAULT_SETS}"
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc$i
  # PMC_CMD overrides the profiled program (default: the MNIST bench), e.g. "bench_resnet.py --steps 2 --warmup 1"
  timeout -s KILL ${PMC_TIMEOUT:-120} rocprofv3 --pmc $set --kernel-trace -d gpurun_out/pmc$i -o run -- python3 ${PMC_CMD:-bench.py --steps 20 --warmup 5 --min_warmup_ms 0 --phases 0} > gpurun_out/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 gpurun_out/pmc$i.log; exit 1; }
  python scripts/pmc_summary.py $(find gpurun_out/pmc$i -name "*.db" | head -1) | tee gpurun_out/pmc$i.txt
  rm -rf gpurun_out/pmc$i
done
