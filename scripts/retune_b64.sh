#!/bin/bash
# Measure the GEMM table entries the batch-64 big-model recipes are missing (existing entries
# kept), then A/B the shipped vs the merged table on those recipes.
export DPC_GEMM_TUNE_OUT=gpurun_out/gemm_tuned_b64.json
rm -f $DPC_GEMM_TUNE_OUT
DPC_GEMM_TUNE=1 scripts/gpu_step.sh "400:rt_fsdp:python -u bench.py --recipe fsdp --steps 1 --warmup 1" \
  "400:rt_ppd:python -u bench.py --recipe pipe_ddp --steps 1 --warmup 1" || exit $?
scripts/gpu_step.sh "200:old_fsdp:python -u bench.py --recipe fsdp --steps 6 --warmup 2" \
  "200:old_ppd:python -u bench.py --recipe pipe_ddp --steps 6 --warmup 2" || exit $?
export DPC_GEMM_TABLE_PATH=$DPC_GEMM_TUNE_OUT
scripts/gpu_step.sh "200:new_fsdp:python -u bench.py --recipe fsdp --steps 6 --warmup 2" \
  "200:new_ppd:python -u bench.py --recipe pipe_ddp --steps 6 --warmup 2"
