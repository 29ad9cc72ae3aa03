#!/bin/bash
# round 5 job 28: same-box A/B of the last three changes (embedding pieces, final-norm dx_set, FFN
# tail bias sums into the gradient) against the tree before them (ab_mid/ = 55be8fa), interleaved
scripts/gpu_step.sh \
  "200:r5_b_new28a:python -u bench.py" \
  "200:r5_b_mid28a:cd ab_mid && python -u bench.py" \
  "200:r5_b_new28b:python -u bench.py" \
  "200:r5_b_mid28b:cd ab_mid && python -u bench.py" \
  "200:r5_b_new28c:python -u bench.py" \
  "200:r5_b_mid28c:cd ab_mid && python -u bench.py"
