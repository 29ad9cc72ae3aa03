#!/bin/bash
# Reference-default config (D=256, S=256, B=64): LayerNorm-backward grid sweep at its shape, GEMM
# table entries for its products (missing signatures measured), then the bench with the new table.
export DPC_GEMM_TUNE_OUT=gpurun_out/gemm_tuned_ref.json
rm -f $DPC_GEMM_TUNE_OUT
scripts/gpu_step.sh "120:ln_grid:python -u bench/ln_grid.py 16320x256,65472x768,65472x1600" \
  "300:rt_ref:env DPC_GEMM_TUNE=1 python -u bench.py --model ref --seq_len 256 --batch_size 64 --steps 2 --warmup 1" \
  "120:ref_old:python -u bench.py --model ref --seq_len 256 --batch_size 64 --steps 50 --warmup 10" \
  "120:ref_new:env DPC_GEMM_TABLE_PATH=gpurun_out/gemm_tuned_ref.json python -u bench.py --model ref --seq_len 256 --batch_size 64 --steps 50 --warmup 10"
