#!/bin/bash
# Full GPU test suite, the GPT-2 GEMM A/B against hipBLASLt, the 1-GPU bench, DMA ablations.
scripts/gpu_step.sh "400:gputests:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "300:ab_gpt2s:python -u bench/gemm_ab.py --shapes gpt2s --impls 22 25 --rounds 3" \
  "300:bench1:python -u bench.py" \
  "120:lab_dma_sq8k:bench/g7lab 8192 8192 8192 nt 5 5 dma" \
  "120:lab_dma_sq8k_nn:bench/g7lab 8192 8192 8192 nn 5 5 dma" \
  "120:lab_dma_upd:bench/g7lab 65536 768 3072 nn 5 20 dma"
