#!/bin/bash
# Round 5: PMC passes over the fp32 MNIST step (MFMA busy, LDS conflicts, waits, bytes).
export PMC_CMD="bench.py --dtype fp32 --steps 20 --warmup 5 --min_warmup_ms 0 --phases 0 --state_steps 0"
bash scripts/gpu_pmc.sh > gpurun_out/r5_f32_pmc.txt 2>&1 || { tail -30 gpurun_out/r5_f32_pmc.txt; exit 1; }
python scripts/pmc_derived.py gpurun_out/r5_f32_pmc.txt
