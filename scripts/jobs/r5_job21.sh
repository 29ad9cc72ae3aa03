#!/bin/bash
# round 5 job 21: the other recipes on the current tree, and FSDP XL on its N > 1 code path
# (--force_dist_path: sharded store, unit-wise AdamW as each reduce-scatter lands) against ab_old/
scripts/gpu_step.sh \
  "400:r5_fsdp_new:python -u bench.py --recipe fsdp --steps 6 --warmup 2" \
  "400:r5_fsdp_old:cd ab_old && python -u bench.py --recipe fsdp --steps 6 --warmup 2" \
  "400:r5_fsdpd_new:python -u bench.py --recipe fsdp --steps 6 --warmup 2 --force_dist_path" \
  "400:r5_fsdpd_old:cd ab_old && python -u bench.py --recipe fsdp --steps 6 --warmup 2 --force_dist_path" \
  "300:r5_pipe_new:python -u bench.py --recipe pipe --steps 6 --warmup 2" \
  "300:r5_pipeddp_new:python -u bench.py --recipe pipe_ddp --steps 6 --warmup 2"
