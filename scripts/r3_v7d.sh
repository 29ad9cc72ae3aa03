#!/bin/bash
# Deferred GELU epilogues (impl 24): numerics, then same-box A/B against the shipped choice
# (i0) and v8 (i21) on the fused-epilogue products; then the --cpu_offload breakdown.
scripts/gpu_step.sh "300:v7d_test:python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k v7d" \
  "400:v7d_ab:python -u bench/gemm_ab.py --shapes fused --impls 20 21 24 --rounds 3" \
  "200:off_none:python -u bench/offload.py --offload 0" \
  "300:off_break:python -u bench/offload.py --breakdown"
