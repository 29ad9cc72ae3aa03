#!/bin/bash
# PMC passes of the v7 GEMM (impl 20) on the GPT-2 small QKV forward (K = 768) and 8192^3 (nt)
set -e
R=$GRAFT_REPO_ROOT
bash scripts/pmc_gemm.sh v7qkv 20 65472 2304 768 nt
bash scripts/pmc_gemm.sh v7sq 20 8192 8192 8192 nt
cd $R
for t in v7qkv v7sq; do for p in a b c; do
  db=$(find gpurun_out/pmc_${t}_$p -name "*.db" | head -1)
  echo "== $t $p"; python3 scripts/pmc_summary.py $db gemm7
done; done > gpurun_out/pmc_v7_summary.txt
rm -rf gpurun_out/pmc_v7qkv_* gpurun_out/pmc_v7sq_*
cat gpurun_out/pmc_v7_summary.txt
