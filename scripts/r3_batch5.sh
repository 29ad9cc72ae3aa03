#!/bin/bash
# Streamlined plain epilogue (buffer stores, scalar row offsets, DPP-masked row trade, alpha 1
# fast path) vs the general path (DPC_G7_DEBUG=16), same box.
scripts/gpu_step.sh "400:gputests:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200:fe_new:python -u bench/gemm_ab.py --shapes gpt2s --impls 20 --rounds 3 --iters 5" \
  "200:fe_old:env DPC_G7_DEBUG=16 python -u bench/gemm_ab.py --shapes gpt2s --impls 20 --rounds 3 --iters 5" \
  "150:b_new:python -u bench.py" "150:b_old:env DPC_G7_DEBUG=16 python -u bench.py" \
  "150:b_new2:python -u bench.py" "150:b_old2:env DPC_G7_DEBUG=16 python -u bench.py" \
  "200:b_fsdp_new:python -u bench.py --recipe fsdp --steps 6 --warmup 2" "200:b_fsdp_old:env DPC_G7_DEBUG=16 python -u bench.py --recipe fsdp --steps 6 --warmup 2"
