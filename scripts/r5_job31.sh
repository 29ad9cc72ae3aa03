#!/bin/bash
# round 5 job 31: the up-projection's fused epilogue with plain (write-back) vs non-temporal
# output stores (DPC_GEMM_NT: the store acknowledgement latency bounds the next tile's counted
# waits), interleaved processes
mkdir -p gpurun_out
for r in 1 2; do
  for nt in 3 0 1 2; do
    echo "== DPC_GEMM_NT=$nt"
    DPC_GEMM_NT=$nt timeout -k 10 120 python -u bench/epi_decomp.py --rounds 3 --iters 10 --only up_plain up_bias up_full || exit $?
  done
done > gpurun_out/r5_nt_ab.log 2>&1
cat gpurun_out/r5_nt_ab.log | grep -v amdgpu.ids
