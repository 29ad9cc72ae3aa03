#!/bin/bash
# round 5 job 4: v9 EPI 1 full-tile fast path (v7 EPI 8 / 9 back to one epilogue copy),
# attention without SLP packing; same-box A/B against ab_old/ (the round-5 start)
scripts/gpu_step.sh \
  "300:r5_t4:python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k 'gemm_v7 or gemm_v9 or attention' tests/test_engines_gpu.py tests/test_native_comm.py -m gpu" \
  "200:r5_d_new2:python -u bench/epi_decomp.py --rounds 5 --iters 10 --only up_plain up_bias up_full dg_full dn_full" \
  "200:r5_d_old2:cd ab_old && python -u bench/epi_decomp.py --rounds 5 --iters 10 --only up_plain up_bias up_full dg_full dn_full" \
  "200:r5_b_new3:python -u bench.py" \
  "200:r5_b_old3:cd ab_old && python -u bench.py" \
  "200:r5_b_new4:python -u bench.py" \
  "200:r5_b_old4:cd ab_old && python -u bench.py"
