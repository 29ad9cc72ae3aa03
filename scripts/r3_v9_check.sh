#!/bin/bash
# v9 (64-deep stages) for plain nt products: GEMM GPU tests, the GPT-2 / XL / square A/B against
# hipBLASLt, the default bench.
scripts/gpu_step.sh "300:gemmtests:python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_table_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "300:ab_gpt2s:python -u bench/gemm_ab.py --shapes gpt2s --impls 22 25 26 --rounds 3" \
  "400:ab_xl:python -u bench/gemm_ab.py --shapes xl --impls 22 25 26 --rounds 3" \
  "300:ab_sq:python -u bench/gemm_ab.py --shapes square --impls 22 25 26 --rounds 3" \
  "200:bench1:python -u bench.py" "200:bench2:DPC_G9=0 python -u bench.py" "200:bench3:python -u bench.py"
