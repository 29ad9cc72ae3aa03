#!/bin/bash
# v8 (2 workgroups / CU) with the second workgroup of each CU phase-shifted (DPC_G8_STAGGER_NS)
# vs the table's choice, on the fused FFN products and the plain GPT-2 small products.
steps=()
for ns in 0 3000 6000; do
  steps+=("200:st8_fused_$ns:env DPC_G8_STAGGER_NS=$ns python -u bench/gemm_ab.py --shapes fused --impls 20 21 --rounds 3 --iters 5")
  steps+=("200:st8_plain_$ns:env DPC_G8_STAGGER_NS=$ns python -u bench/gemm_ab.py --shapes gpt2s --impls 20 21 --rounds 3 --iters 5")
done
scripts/gpu_step.sh "${steps[@]}"
