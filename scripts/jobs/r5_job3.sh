#!/bin/bash
# round 5 job 3: check-free, act-specialised full-tile epilogues (v9 EPI 1, v7 EPI 8 / 9),
# attention without SLP packing / with the in-place rescale: numerics, then a same-box A/B
# against the previous commit (ab_old/); plus the device-seed dropout graph and unit-wise FSDP
scripts/gpu_step.sh \
  "600:r5_t3:python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k 'gemm or attention' -m gpu" \
  "300:r5_t3b:python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engines_gpu.py tests/test_native_comm.py tests/test_model_gpu.py -m gpu" \
  "200:r5_d_new1:python -u bench/epi_decomp.py --rounds 5 --iters 10 --only up_plain up_bias up_full dg_full dn_full" \
  "200:r5_d_old1:cd ab_old && python -u bench/epi_decomp.py --rounds 5 --iters 10 --only up_plain up_bias up_full dg_full dn_full" \
  "200:r5_a_new1:python -u bench/attn_time.py" \
  "200:r5_a_old1:cd ab_old && python -u bench/attn_time.py" \
  "200:r5_b_new1:python -u bench.py" \
  "200:r5_b_old1:cd ab_old && python -u bench.py" \
  "200:r5_b_new2:python -u bench.py" \
  "200:r5_b_old2:cd ab_old && python -u bench.py"
