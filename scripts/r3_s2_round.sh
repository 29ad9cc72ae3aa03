#!/bin/bash
# Mid-session round check: the driver's GPU tiers + the four recipe benches, the GPT-2 small and
# XL products against hipBLASLt, and a rocprofv3 kernel table of the default (DDP) step.
bash scripts/round_check.sh || exit $?
scripts/gpu_step.sh "300:ab_gpt2s:python -u bench/gemm_ab.py --shapes gpt2s --impls 22 25 --rounds 3" \
  "400:ab_xl:python -u bench/gemm_ab.py --shapes xl --impls 22 25 --rounds 3" \
  "300:ab_sq:python -u bench/gemm_ab.py --shapes square --impls 22 25 --rounds 3" || exit $?
bash scripts/prof_bench.sh s2_ddp --recipe ddp
