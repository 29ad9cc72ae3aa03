#!/bin/bash
# round 5 job 5: v7 EPI 8 / 9 epilogues without branches (act by select, next pair's operand
# read ahead, bounded buffer stores): numerics, same-box A/B against ab_old/
scripts/gpu_step.sh \
  "300:r5_t5:python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k 'gemm' tests/test_model_gpu.py tests/test_fp32_gpu.py -m gpu" \
  "200:r5_d_new3:python -u bench/epi_decomp.py --rounds 5 --iters 10 --only up_plain up_full dg_full dn_full" \
  "200:r5_d_old3:cd ab_old && python -u bench/epi_decomp.py --rounds 5 --iters 10 --only up_plain up_full dg_full dn_full" \
  "200:r5_b_new5:python -u bench.py" \
  "200:r5_b_old5:cd ab_old && python -u bench.py" \
  "200:r5_b_new6:python -u bench.py" \
  "200:r5_b_old6:cd ab_old && python -u bench.py"
