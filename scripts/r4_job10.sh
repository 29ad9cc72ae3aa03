#!/bin/bash
# the fused-epilogue FFN products on v8 (256 x 128 tiles, two workgroups per CU: one's epilogue
# beside the other's MFMAs) against the table (v9 EPI 1 / v7 EPI 8)
scripts/gpu_step.sh "300:warm:python -u scripts/warm.py" \
  "300:ab_fused_v8:python -u bench/gemm_ab.py --shapes fused --impls 21 26 10" || exit $?
