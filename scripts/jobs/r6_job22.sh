#!/bin/bash
# round 6 job 22: head_dim 32 forward (the reference CLI default model: D 256, 8 heads of 32,
# S 256): the shipped variant 2 against the pair streams 6 (fwd2) and 9 (fwd3)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for shape in "--N 64 --S 255 --H 8 --hd 32" "--N 64 --S 1023 --H 8 --hd 32"; do
  for r in 1 2; do
    for v in 2 6 9; do
      echo -n "$shape var $v: "; DPC_ATTN_VAR=$v,2 timeout -k 10 120 python -u bench/attn_time.py $shape --rounds 5 --iters 20 2>/dev/null \
        | grep '^{' || exit 4
    done
  done
done | tee gpurun_out/r6_attn_hd32.log
