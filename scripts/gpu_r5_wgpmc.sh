#!/bin/bash
# Round 5: PMC passes over one ResNet-50 weight-gradient GEMM (l3 1x1 256->1024 at batch 128).
export PMC_CMD="scripts/debug/gemm_probe.py --match l3.1x1.256-1024 --only wgrad --torch 0 --iters 20"
export PMC_SETS="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE;SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_INSTS_VMEM SQ_INSTS_MFMA;SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS TCC_HIT_sum TCC_MISS_sum;FETCH_SIZE"
bash scripts/gpu_pmc.sh > gpurun_out/r5_wg_pmc.txt 2>&1 || { tail -30 gpurun_out/r5_wg_pmc.txt; exit 1; }
cat gpurun_out/r5_wg_pmc.txt
