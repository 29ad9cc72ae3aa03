#!/bin/bash
# v7 persistent-grid start stagger: auto (iNN) vs off (iNNs0) vs forced sizes, then the benches.
scripts/gpu_step.sh \
  "300:st_s:python -u bench/gemm_ab.py --shapes gpt2s --impls 20 19 --stagger 0 2 4 8 --rounds 3 --iters 5" \
  "300:st_xl:python -u bench/gemm_ab.py --shapes xl --impls 20 --stagger 0 4 --rounds 3 --iters 5" \
  "200:b_on:python -u bench.py" \
  "200:b_off:env DPC_G7_STAGGER=0 python -u bench.py" \
  "200:b_on2:python -u bench.py" \
  "200:b_off2:env DPC_G7_STAGGER=0 python -u bench.py"
