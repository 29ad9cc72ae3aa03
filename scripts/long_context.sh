#!/bin/bash
# SURVEY §5.7 long context on one MI355X: the new long-S numerics tests, then GPT-2 small
# training throughput at a fixed 64K tokens/step as the context grows 1K -> 8K, then a kernel
# profile at 8K.  Results in gpurun_out/lc_*.
scripts/gpu_step.sh \
  "240:lc_tests:python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k 'long_context'" \
  "150:lc_s2048:python -u bench.py --seq_len 2048 --batch_size 32 --steps 10 --warmup 3" \
  "150:lc_s4096:python -u bench.py --seq_len 4096 --batch_size 16 --steps 10 --warmup 3" \
  "150:lc_s8192:python -u bench.py --seq_len 8192 --batch_size 8 --steps 10 --warmup 3" \
  "400:lc_prof:bash scripts/prof_bench.sh s8192 --seq_len 8192 --batch_size 8"
