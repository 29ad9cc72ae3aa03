#!/bin/bash
# Per-GPU batch of the big-model recipes at the reference default (--batch_size 64) vs 32 / 48
scripts/gpu_step.sh \
  "200:f32:python -u bench.py --recipe fsdp --steps 6 --warmup 2" \
  "200:f48:python -u bench.py --recipe fsdp --steps 6 --warmup 2 --batch_size 48" \
  "250:f64:python -u bench.py --recipe fsdp --steps 6 --warmup 2 --batch_size 64" \
  "200:l64:python -u bench.py --recipe pipe_ddp --steps 6 --warmup 2 --batch_size 64" \
  "200:m96:python -u bench.py --recipe pipe --steps 6 --warmup 2 --batch_size 96"
