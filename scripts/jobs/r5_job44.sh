#!/bin/bash
# round 5 job 44: attention PMC on the final kernels (wait / issue / instruction mix)
mkdir -p gpurun_out
timeout -k 10 400 bash scripts/pmc_attn_all.sh > gpurun_out/r5_pmc_attn.log 2>&1 || { tail -20 gpurun_out/r5_pmc_attn.log; exit 1; }
cat gpurun_out/pmc_attn_summary.txt
