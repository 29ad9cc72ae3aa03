#!/bin/bash
# round 5 job 70: plain stores for small bf16 GEMM outputs (DPC_GEMM_NT_SMALL_MB 0 / 128 / 256),
# interleaved in the step
mkdir -p gpurun_out
for r in 1 2 3; do
  for mb in 0 128 256; do
    echo "== small $mb"; DPC_GEMM_NT_SMALL_MB=$mb timeout -k 10 200 python -u bench.py 2>&1 | grep -v amdgpu.ids | grep -o '"value": [0-9.]*' || exit 1
  done
done
