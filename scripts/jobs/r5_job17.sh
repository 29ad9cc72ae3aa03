#!/bin/bash
# round 5 job 17: pipeline micro-batch count sweep on the one-GPU stage proxy:
# per-token time of M micro-batches of mb sequences against one full batch, at a fixed batch
# per pipeline (PP=8 medium: 512 sequences; PP=2 large: 128)
mkdir -p gpurun_out/r5_pp
for cfg in "gpt2-medium 8 16 32" "gpt2-medium 8 32 16" "gpt2-medium 8 64 8" "gpt2-large 2 4 32" "gpt2-large 2 8 16" "gpt2-large 2 16 8"; do
  set -- $cfg
  echo "== $cfg"
  timeout -k 10 240 python -u bench/pp_stage_proxy.py --model $1 --pp $2 --micro $3 --mb $4 --steps 3 --warmup 1 \
    --json gpurun_out/r5_pp/pp$2_$1_m$3.json > gpurun_out/r5_pp/pp$2_$1_m$3.log 2>&1 || exit $?
  tail -1 gpurun_out/r5_pp/pp$2_$1_m$3.log
done
