#!/bin/bash
# round 5 job 13: cross-entropy kernel with the per-logit VALU cut (ce_kernel2), AdamW with two
# groups in flight per thread + nt accesses; numerics, CE timing, same-box bench A/B
scripts/gpu_step.sh \
  "600:r5_t13:python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_engines_gpu.py -m gpu" \
  "200:r5_ce13:python -u bench/ce_one.py" \
  "200:r5_b_new13:python -u bench.py" \
  "200:r5_b_old13:cd ab_old && python -u bench.py" \
  "200:r5_b_new13b:python -u bench.py" \
  "200:r5_b_old13b:cd ab_old && python -u bench.py"
