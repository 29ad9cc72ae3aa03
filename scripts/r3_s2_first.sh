#!/bin/bash
# Session 2 of round 3, first GPU call: the v7 main-loop ablation ladder (bench/g7lab), v7d
# numerics + same-box A/B of the deferred epilogues, the default 1-GPU bench.
scripts/gpu_step.sh "120:lab_sq8k:bench/g7lab 8192 8192 8192 nt 5 5" \
  "120:lab_qkv:bench/g7lab 65536 2304 768 nt 5 20" \
  "120:lab_sq8k_nn:bench/g7lab 8192 8192 8192 nn 5 5" \
  "300:v7d_test:python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k v7d" \
  "400:v7d_ab:python -u bench/gemm_ab.py --shapes fused --impls 20 21 24 --rounds 3" \
  "300:bench1:python -u bench.py"
