#!/bin/bash
# round 5 job 7: kernel table of the DDP step after the epilogue work; attention timings
scripts/gpu_step.sh \
  "400:r5_prof7:scripts/prof_bench.sh r5a" \
  "200:r5_attn7:python -u bench/attn_time.py"
