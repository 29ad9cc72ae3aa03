#!/bin/bash
# reference-default config after the LN-backward grid rule + table entries; LN / table tests
scripts/gpu_step.sh "300:t_ln:python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_table_gpu.py -x -q --timeout 120 --timeout-method thread -k 'layernorm or table'" \
  "120:ref_a:python -u bench.py --model ref --seq_len 256 --batch_size 64 --steps 50 --warmup 10" \
  "120:ref_b:python -u bench.py --model ref --seq_len 256 --batch_size 64 --steps 50 --warmup 10" \
  "150:b_ddp:python -u bench.py"
