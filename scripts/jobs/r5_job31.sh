#!/bin/bash
# round 5 job 31b: the fused up-projection epilogue stores with cache-policy variants (DPC_GEMM_NT 3 + 4 x pol:
# output stores (DPC_GEMM_NT: the store acknowledgement latency bounds the next tile's counted
# waits), interleaved processes
mkdir -p gpurun_out
for r in 1 2 3; do
  for nt in 3 11 15; do
    echo "== DPC_GEMM_NT=$nt"
    DPC_GEMM_NT=$nt timeout -k 10 120 python -u bench/epi_decomp.py --rounds 5 --iters 10 --only up_plain up_bias up_full || exit $?
  done
done > gpurun_out/r5_nt_ab.log 2>&1
cat gpurun_out/r5_nt_ab.log | grep -v amdgpu.ids
