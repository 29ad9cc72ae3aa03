#!/bin/bash
# A/B of the attention kernel variants (DPC_ATTN_VAR) at the GPT-2 small shape.
for hd in ${HDS:-64 32}; do
  for v in ${VARS:-0 1 2 3}; do
    DPC_ATTN_VAR=$v,$v timeout -k 5 60 python -u bench/attn_one.py --N 64 --S 1023 --H 12 --hd $hd --iters 10 | sed "s/^/var$v /" || exit $?
    if [ "$v" != 4 ]; then DPC_ATTN_VAR=$v,$v timeout -k 5 60 python -u bench/attn_one.py --N 64 --S 1023 --H 12 --hd $hd --iters 10 --bwd | sed "s/^/var$v /" || exit $?; fi
  done
done
