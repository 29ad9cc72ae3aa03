#!/bin/bash
# GPT-2 small tokens/s vs per-GPU batch on one MI355X (ours), plus the stock-PyTorch
# reference-default recipe (manual attention + torch.compile) at the reference's default
# per-rank batch of 64 (main-ddp.py argparse).
scripts/gpu_step.sh "150:bs32:python -u bench.py --batch_size 32" \
  "150:bs48:python -u bench.py --batch_size 48" \
  "150:bs64:python -u bench.py --batch_size 64" \
  "200:bs96:python -u bench.py --batch_size 96" \
  "400:stock64:python -u bench/baseline_torch.py --compile --batch_size 64 --steps 10 --warmup 3" \
  "400:stock64sdpa:python -u bench/baseline_torch.py --compile --sdpa --batch_size 64 --steps 10 --warmup 3"
