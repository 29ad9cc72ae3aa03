#!/bin/bash
# round 5 job 9: dK / dV causal zeroing in place, on diagonal sub-blocks only
scripts/gpu_step.sh \
  "500:r5_t9:python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp32_gpu.py -m gpu" \
  "200:r5_a_new9:python -u bench/attn_time.py" \
  "200:r5_a_old9:cd ab_old && python -u bench/attn_time.py" \
  "200:r5_a_new9b:python -u bench/attn_time.py" \
  "200:r5_a_old9b:cd ab_old && python -u bench/attn_time.py"
