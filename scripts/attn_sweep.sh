#!/bin/bash
# Attention fwd / bwd throughput at equal tokens (N*S = 64K) over the sequence length.
for x in "64 1023" "32 2047" "16 4095" "8 8191"; do
  set -- $x
  timeout -k 5 60 python -u bench/attn_one.py --N $1 --S $2 --H 12 --hd ${HD:-64} --iters 20 || exit $?
  timeout -k 5 60 python -u bench/attn_one.py --N $1 --S $2 --H 12 --hd ${HD:-64} --iters 20 --bwd || exit $?
done
