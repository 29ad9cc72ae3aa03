#!/bin/bash
# LM-head / layer weight-gradient products (tn, f32 out): implementation x forced split-K count.
run() { timeout -k 5 90 python -u bench/gemm_one.py --layout tn --iters 10 "$@" 2>&1 | grep TF/s || exit 1; }
for shape in "50304 768 65472" "50304 1600 32736" "2304 768 65472" "3072 768 65472"; do
  set -- $shape
  run --M $1 --N $2 --K $3 --impl -1
  run --M $1 --N $2 --K $3 --impl 12
  for sp in 1 2 3 4 6; do run --M $1 --N $2 --K $3 --impl 20 --splits $sp; done
done
