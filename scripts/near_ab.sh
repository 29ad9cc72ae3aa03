#!/bin/bash
# nearest-signature GEMM table lookup: long-context GPT-2 small (M = 8 x 8191 etc. are not in the
# table) with exact-only lookup vs nearest, alternating; then the default bench (unchanged keys).
for rep in 1 2; do
  for v in 0 1; do
    scripts/gpu_step.sh "150:s8192_n${v}_$rep:env DPC_GEMM_NEAR=$v python -u bench.py --seq_len 8192 --batch_size 8 --steps 10 --warmup 3" \
      "150:s4096_n${v}_$rep:env DPC_GEMM_NEAR=$v python -u bench.py --seq_len 4096 --batch_size 16 --steps 10 --warmup 3" \
      "150:s2048_n${v}_$rep:env DPC_GEMM_NEAR=$v python -u bench.py --seq_len 2048 --batch_size 32 --steps 10 --warmup 3" || exit $?
  done
done
