#!/bin/bash
# The reference's own CLI default model (D=256, 8 x 32 heads, 8 layers, sequence_length 256,
# batch 64): this framework (bench.py, HIP-graph step) vs stock PyTorch (reference math + compile,
# and SDPA + compile), one MI355X.
scripts/gpu_step.sh \
  "200:ours_ref:python -u bench.py --model ref --seq_len 256 --batch_size 64 --steps 50 --warmup 10" \
  "400:stock_ref_compile:python -u bench/baseline_torch.py --model ref --batch_size 64 --seq_len 256 --steps 50 --warmup 10 --compile" \
  "400:stock_ref_sdpa_compile:python -u bench/baseline_torch.py --model ref --batch_size 64 --seq_len 256 --steps 50 --warmup 10 --compile --sdpa"
