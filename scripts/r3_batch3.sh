#!/bin/bash
# Round-3 batch 3: attention 5-slot rings (fwd var 9, dQ var 4) numerics + timing A/B;
# v7 epilogue ablations (1 = no epilogue, 4 = epilogue VALU without stores).
steps=("300:attn_t9:env DPC_ATTN_VAR=9,4 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k attention")
for rep in 1 2; do
  for v in 6,1 9,4; do
    steps+=("60:attn_f_${v/,/_}_$rep:env DPC_ATTN_VAR=$v python bench/attn_one.py --N 64 --iters 20")
    steps+=("60:attn_b_${v/,/_}_$rep:env DPC_ATTN_VAR=$v python bench/attn_one.py --N 64 --iters 10 --bwd")
  done
done
for d in 0 1 4; do
  steps+=("200:epi_dbg$d:env DPC_G7_DEBUG=$d python -u bench/gemm_ab.py --shapes gpt2s --impls 20 --rounds 3 --iters 5")
done
steps+=("150:b_ddp_attn94:env DPC_ATTN_VAR=9,4 python -u bench.py" "150:b_ddp_attn61:env DPC_ATTN_VAR=6,1 python -u bench.py")
scripts/gpu_step.sh "${steps[@]}"
