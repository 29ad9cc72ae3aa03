#!/bin/bash
# v9 epilogue experiments on the GPT-2-small forward shapes (bench/g7lab "epi" set)
scripts/gpu_step.sh "120:lab_qkv:bench/g7lab 65536 2304 768 nt 5 10 epi" \
  "120:lab_up:bench/g7lab 65536 3072 768 nt 5 10 epi" \
  "120:lab_lm:bench/g7lab 65536 49152 768 nt 3 3 epi" \
  "120:lab_sq:bench/g7lab 8192 8192 8192 nt 3 5 epi"
