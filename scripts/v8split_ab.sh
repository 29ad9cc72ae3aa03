#!/bin/bash
# v8 (256 x 128 tiles, 2 WG / CU) with workspace-slab split-K for the weight gradients: GEMM tests,
# then v7 (i20) vs v8 (i21) on the GPT-2 XL and GPT-2 small weight-gradient shapes.
scripts/gpu_step.sh "300:t_gemm:python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k 'split or v6_v7'" \
  "300:ab_xl:python -u bench/gemm_ab.py --shapes xl --only xl_w_qkv xl_w_out xl_w_up xl_w_down xl_w_lm --impls 20 21 --rounds 3 --iters 5"
