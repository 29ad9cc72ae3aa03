#!/bin/bash
# Round-4 opening check on one MI355X: the DDP bench, its kernel table, the GPT-2-small GEMM
# A/B against hipBLASLt and the attention kernels at the bench shape.
scripts/gpu_step.sh "150:b_ddp:python -u bench.py" \
  "300:gemm_ab:python -u bench/gemm_ab.py --shapes gpt2s --rounds 3" \
  "60:attn_fwd:python -u bench/attn_one.py --N 64 --S 1023 --H 12 --iters 20" \
  "60:attn_bwd:python -u bench/attn_one.py --N 64 --S 1023 --H 12 --iters 20 --bwd" || exit $?
bash scripts/prof_bench.sh r4_ddp
