#!/bin/bash
# v7 epilogue stores: chip-bandwidth-bound or per-CU bound?  8 = every other workgroup skips its
# stores (half the chip-wide store traffic, the same per storing CU).
steps=()
for d in 0 8 4 0 8 4; do
  steps+=("200:epi2_dbg$d:env DPC_G7_DEBUG=$d python -u bench/gemm_ab.py --shapes gpt2s --only qkv_fwd lm_fwd up_fwd out_fwd --impls 20 --rounds 3 --iters 5")
done
scripts/gpu_step.sh "${steps[@]}"
