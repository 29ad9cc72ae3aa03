#!/bin/bash
# Few-row GEMV kernel: numerics + decode tests, then greedy-decode latency with the library
# product (DPC_GEMV=0) vs the kernel, GPT-2 small and XL.
scripts/gpu_step.sh \
  "200:t_gemv:python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -k 'gemv or decode or generate or kv or graph_decoder or last_only'" \
  "200:g_s_lib:env DPC_GEMV=0 python -u bench/generate.py --model gpt2-small" \
  "200:g_s_new:python -u bench/generate.py --model gpt2-small" \
  "300:g_xl_lib:env DPC_GEMV=0 python -u bench/generate.py --model gpt2-xl" \
  "300:g_xl_new:python -u bench/generate.py --model gpt2-xl"
