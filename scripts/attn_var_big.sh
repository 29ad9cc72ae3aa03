#!/bin/bash
# attention kernel variants (DPC_ATTN_VAR=<fwd>,<bwd>) at the big-model shapes (N=64, S=1023):
# H = 16 (medium), 20 (large), 25 (XL), hd 64
for H in 12 16 20 25; do
  for v in 0 1 2 3; do
    echo -n "H=$H bwd var $v: "
    DPC_ATTN_VAR=6,$v timeout -k 10 60 python -u bench/attn_one.py --N 64 --S 1023 --H $H --iters 10 --bwd 2>/dev/null | tail -1 || exit $?
  done
  for v in 0 2 5 6; do
    echo -n "H=$H fwd var $v: "
    DPC_ATTN_VAR=$v,1 timeout -k 10 60 python -u bench/attn_one.py --N 64 --S 1023 --H $H --iters 10 2>/dev/null | tail -1 || exit $?
  done
done
