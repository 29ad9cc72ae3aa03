#!/bin/bash
# round 5 job 54: GEMM PMC (MFMA busy, waits, LDS bank conflicts, L2 hit) of the step's split-K
# weight gradient (up projection) and plain input gradient (up projection)
mkdir -p gpurun_out
bash scripts/pmc_gemm.sh dw -1 3072 768 65472 tn > gpurun_out/r5_pmc_gemm.log 2>&1 || { tail -20 gpurun_out/r5_pmc_gemm.log; exit 1; }
bash scripts/pmc_gemm.sh dx -1 65472 768 3072 nn >> gpurun_out/r5_pmc_gemm.log 2>&1 || { tail -20 gpurun_out/r5_pmc_gemm.log; exit 1; }
for t in dw dx; do for p in a b c; do echo "== $t $p"; python3 scripts/pmc_summary.py $(find gpurun_out/pmc_${t}_${p} -name "*.db" | head -1) gemm; done; done > gpurun_out/r5_pmc_gemm_summary.txt
cat gpurun_out/r5_pmc_gemm_summary.txt
rm -rf gpurun_out/pmc_dw_* gpurun_out/pmc_dx_*
