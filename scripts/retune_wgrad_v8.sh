#!/bin/bash
# Re-measure every weight-gradient table entry (mm:f) now that v8 (impl 21) splits K too, over
# the four recipes (and the reference-default model), then A/B shipped vs re-measured table.
cp scripts/gemm_table_no_mm.json gpurun_out/gemm_tuned_wg.json
export DPC_GEMM_TUNE_OUT=gpurun_out/gemm_tuned_wg.json
export DPC_GEMM_TABLE_PATH=gpurun_out/gemm_tuned_wg.json
DPC_GEMM_TUNE=1 scripts/gpu_step.sh "300:rt_ddp:python -u bench.py --steps 1 --warmup 1" \
  "400:rt_fsdp:python -u bench.py --recipe fsdp --steps 1 --warmup 1" \
  "300:rt_pipe:python -u bench.py --recipe pipe --steps 1 --warmup 1" \
  "400:rt_ppd:python -u bench.py --recipe pipe_ddp --steps 1 --warmup 1" \
  "300:rt_ref:python -u bench.py --model ref --seq_len 256 --batch_size 64 --steps 1 --warmup 1" || exit $?
unset DPC_GEMM_TUNE_OUT DPC_GEMM_TABLE_PATH
for rep in 1 2; do
  scripts/gpu_step.sh "150:o_ddp_$rep:python -u bench.py" "200:o_fsdp_$rep:python -u bench.py --recipe fsdp --steps 6 --warmup 2" \
    "200:o_pipe_$rep:python -u bench.py --recipe pipe --steps 6 --warmup 2" "200:o_ppd_$rep:python -u bench.py --recipe pipe_ddp --steps 6 --warmup 2" || exit $?
  DPC_GEMM_TABLE_PATH=gpurun_out/gemm_tuned_wg.json scripts/gpu_step.sh "150:n_ddp_$rep:python -u bench.py" "200:n_fsdp_$rep:python -u bench.py --recipe fsdp --steps 6 --warmup 2" \
    "200:n_pipe_$rep:python -u bench.py --recipe pipe --steps 6 --warmup 2" "200:n_ppd_$rep:python -u bench.py --recipe pipe_ddp --steps 6 --warmup 2" || exit $?
done
