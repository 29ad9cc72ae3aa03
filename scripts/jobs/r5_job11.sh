#!/bin/bash
# round 5 job 11: the FFN tail (down-projection bias / act' / dropout backward) fused into the
# consuming LayerNorm backward; numerics, recipes, same-box bench A/B against ab_old/
scripts/gpu_step.sh \
  "600:r5_t11:python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_engines_gpu.py -m gpu" \
  "200:r5_b_new11:python -u bench.py" \
  "200:r5_b_old11:cd ab_old && python -u bench.py" \
  "200:r5_b_new11b:python -u bench.py" \
  "200:r5_b_old11b:cd ab_old && python -u bench.py"
