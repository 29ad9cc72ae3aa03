#!/bin/bash
# GEMM GPU tests, GPT-2 A/B vs hipBLASLt, bench, and a rocprofv3 kernel table of the DDP step.
scripts/gpu_step.sh "300:gemmtests:python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_table_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "300:ab_gpt2s:python -u bench/gemm_ab.py --shapes gpt2s --impls 22 25 --rounds 3" \
  "300:bench1:python -u bench.py" \
  "400:prof:scripts/prof_bench.sh ddp"
