#!/bin/bash
# v5 (impl 12) and hipBLASLt-sized squares vs the GPT-2 weight-gradient shape, three layouts.
for lay in nt nn tn; do
  for sz in 4096 8192; do
    timeout -k 5 60 python3 bench/gemm_one.py --M $sz --N $sz --K $sz --layout $lay --impl 12 --iters 10 || exit $?
  done
done
timeout -k 5 60 python3 bench/gemm_one.py --M 3072 --N 768 --K 65472 --layout tn --impl 12 --iters 10
timeout -k 5 60 python3 bench/gemm_one.py --M 3072 --N 768 --K 65472 --layout tn --impl -1 --iters 10
