#!/bin/bash
# Re-measure only the weight-gradient (mm, f32) entries of the GEMM table (after the v7
# workspace split-K), every other entry taken from the table; then bench all recipes with it.
export DPC_BLAS_PLAIN=0
export DPC_GEMM_TUNE_OUT=gpurun_out/gemm_tuned_wgrad.json
rm -f $DPC_GEMM_TUNE_OUT
cp scripts/gemm_table_no_wgrad.json gpurun_out/gemm_table_in.json
DPC_GEMM_TABLE_PATH=gpurun_out/gemm_table_in.json DPC_GEMM_TUNE=1 scripts/gpu_step.sh \
  "400:rt_ddp:python -u bench.py --steps 2 --warmup 2" \
  "500:rt_fsdp:python -u bench.py --recipe fsdp --steps 2 --warmup 2" \
  "500:rt_pipe:python -u bench.py --recipe pipe --steps 2 --warmup 2" \
  "500:rt_ppd:python -u bench.py --recipe pipe_ddp --steps 2 --warmup 2" || exit $?
export DPC_GEMM_TABLE_PATH=$DPC_GEMM_TUNE_OUT
scripts/gpu_step.sh "200:n_ddp:python -u bench.py" \
  "300:n_fsdp:python -u bench.py --recipe fsdp --steps 8 --warmup 3" \
  "300:n_pipe:python -u bench.py --recipe pipe --steps 8 --warmup 3" \
  "300:n_ppd:python -u bench.py --recipe pipe_ddp --steps 8 --warmup 3"
