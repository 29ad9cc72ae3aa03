#!/bin/bash
# round 5 job 1: health of the round-4 tree on a fresh box + the fused-epilogue decomposition
scripts/gpu_step.sh \
  "240:r5_decomp:python -u bench/epi_decomp.py --rounds 5 --iters 10" \
  "200:r5_bench1:python -u bench.py" \
  "200:r5_bench2:python -u bench.py"
