#!/bin/bash
# Re-entry check on a fresh box (driver's tiers + the four recipe benches) and the GPT-2 XL
# plain-product A/B (dpc table choice vs v7/v8 impls vs hipBLASLt).
bash scripts/round_check.sh && \
scripts/gpu_step.sh "300:gemm_xl:python -u bench/gemm_ab.py --shapes xl --impls 16 19 20 21 12 --rounds 3 --iters 5"
