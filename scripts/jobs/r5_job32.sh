#!/bin/bash
# round 5 job 32: every v7 / v9 epilogue store with a cache-policy variant (DPC_GEMM_NT = 3 + 4 x
# pol: 0 nt, 2 sc1 nt, 3 sc0 sc1 nt), interleaved processes; then the DDP bench per policy
mkdir -p gpurun_out
for r in 1 2; do
  for nt in 3 11 15; do
    echo "== DPC_GEMM_NT=$nt"
    DPC_GEMM_NT=$nt timeout -k 10 150 python -u bench/epi_decomp.py --rounds 3 --iters 10 \
      --only up_plain up_full dg_plain dg_full dn_plain_f32 dn_full || exit $?
  done
done > gpurun_out/r5_pol_ab.log 2>&1
for r in 1 2; do
  for nt in 3 11 15; do
    echo "== bench DPC_GEMM_NT=$nt"
    DPC_GEMM_NT=$nt timeout -k 10 200 python -u bench.py || exit $?
  done
done >> gpurun_out/r5_pol_ab.log 2>&1
grep -v amdgpu.ids gpurun_out/r5_pol_ab.log | cut -c1-120
