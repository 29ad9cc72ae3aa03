#!/bin/bash
# Weight-gradient products (tn, f32 out): table choice, v5, v7 with automatic / forced split-K
# (DPC_GEMM_WS_MB=0: the f32-atomic split instead of the workspace slabs).
run() { timeout -k 5 90 python -u bench/gemm_one.py --layout tn --iters 10 "$@" 2>&1 | grep TF/s || exit 1; }
for shape in ${SHAPES:-"50304 768 65472" "50304 1600 32736" "2304 768 65472" "3072 768 65472" "768 768 65472" "4800 1600 32736" "6400 1600 32736" "1600 1600 32736"}; do
  set -- $shape
  run --M $1 --N $2 --K $3 --impl -1
  run --M $1 --N $2 --K $3 --impl 12
  run --M $1 --N $2 --K $3 --impl 20
  DPC_GEMM_WS_MB=0 run --M $1 --N $2 --K $3 --impl 20 | sed 's/^/atomics /'
  for sp in ${SPLITS:-2 3 4 6 8}; do run --M $1 --N $2 --K $3 --impl 20 --splits $sp; done
done
