#!/bin/bash
# Round 2: re-measure the GEMM table with the v7 candidates, library path off, over the four
# bench recipes -> gpurun_out/gemm_tuned_r2.json; then bench every recipe with it.
export DPC_BLAS_PLAIN=0
export DPC_GEMM_TUNE_OUT=gpurun_out/gemm_tuned_r2.json
rm -f $DPC_GEMM_TUNE_OUT
DPC_GEMM_TABLE=0 DPC_GEMM_TUNE=1 scripts/gpu_step.sh "400:rt_ddp:python -u bench.py --steps 2 --warmup 2" \
  "500:rt_fsdp:python -u bench.py --recipe fsdp --steps 2 --warmup 2" \
  "500:rt_pipe:python -u bench.py --recipe pipe --steps 2 --warmup 2" \
  "500:rt_ppd:python -u bench.py --recipe pipe_ddp --steps 2 --warmup 2" || exit $?
export DPC_GEMM_TABLE_PATH=$DPC_GEMM_TUNE_OUT
scripts/gpu_step.sh "200:n_ddp:python -u bench.py" \
  "300:n_fsdp:python -u bench.py --recipe fsdp --steps 6 --warmup 2" \
  "300:n_pipe:python -u bench.py --recipe pipe --steps 6 --warmup 2" \
  "300:n_ppd:python -u bench.py --recipe pipe_ddp --steps 6 --warmup 2"
