#!/bin/bash
# Forward-attention ablations (DPC_ATTN_ABL, timing only) at the GPT-2 small shape.
for a in ${ABLS:-0 1 2 6 7 32 33 39 64}; do
  DPC_ATTN_ABL=$a timeout -k 5 60 python -u bench/attn_one.py --N 64 --S 1023 --H 12 --hd 64 --iters 20 | sed "s/^/abl$a /" || exit $?
done
