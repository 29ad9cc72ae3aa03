#!/bin/bash
# round 5 job 27: embedding backward pieces of 8 rows, final-norm backward without the dx zero
# fill, FFN tail bias sums straight into the gradient; numerics + same-box bench A/B
scripts/gpu_step.sh \
  "600:r5_t27:python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_engines_gpu.py -m gpu" \
  "200:r5_b_new27:python -u bench.py" \
  "200:r5_b_old27:cd ab_old && python -u bench.py" \
  "200:r5_b_new27b:python -u bench.py" \
  "200:r5_b_old27b:cd ab_old && python -u bench.py"
