#!/bin/bash
# round 5 job 2: the whole-line v9 EPI 1 epilogue, head_dim 128 attention, the split GEMM build
scripts/gpu_step.sh \
  "600:r5_t2:python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k 'v9_forward_epilogue or attention or test_gemm_v7' tests/test_fp32_gpu.py tests/test_model_gpu.py -m gpu" \
  "240:r5_decomp2:python -u bench/epi_decomp.py --rounds 5 --iters 10 --only up_plain up_bias up_bias_r4 up_full up_full_r4 up_full_tab dg_full dn_full" \
  "200:r5_bench3:python -u bench.py" \
  "200:r5_bench4:python -u bench.py"
