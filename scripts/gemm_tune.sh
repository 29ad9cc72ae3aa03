#!/bin/bash
# Measure the per-shape GEMM implementation table (ops/gemm_tuned.json) on one MI355X over
# the four bench recipes; the merged table lands in gpurun_out/gemm_tuned.json.
export DPC_GEMM_TUNE=1 DPC_GEMM_TUNE_OUT=gpurun_out/gemm_tuned.json
scripts/gpu_step.sh "200:t_ddp:python -u bench.py --steps 5 --warmup 2" \
  "300:t_fsdp:python -u bench.py --recipe fsdp --batch_size 16 --steps 3 --warmup 2" \
  "300:t_pipe:python -u bench.py --recipe pipe --steps 3 --warmup 2" \
  "300:t_ppd:python -u bench.py --recipe pipe_ddp --batch_size 16 --steps 3 --warmup 2"
