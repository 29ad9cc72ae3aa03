#!/bin/bash
# Re-measure the whole GEMM table with the split-interleave v7 (SCHED 6 on mn-major operands,
# impl 25 candidate), A/B old vs new table on the four recipe benches (same box, two
# alternations), then the --cpu_offload stage breakdown.
export DPC_GEMM_TUNE_OUT=gpurun_out/gemm_tuned_r3b.json
rm -f $DPC_GEMM_TUNE_OUT
DPC_GEMM_TABLE=0 DPC_GEMM_TUNE=1 scripts/gpu_step.sh "300:rt_ddp:python -u bench.py --steps 1 --warmup 1" \
  "400:rt_fsdp:python -u bench.py --recipe fsdp --steps 1 --warmup 1" \
  "300:rt_pipe:python -u bench.py --recipe pipe --steps 1 --warmup 1" \
  "400:rt_ppd:python -u bench.py --recipe pipe_ddp --steps 1 --warmup 1" || exit $?
for rep in 1 2; do
  scripts/gpu_step.sh "150:old_ddp_$rep:python -u bench.py" "200:old_fsdp_$rep:python -u bench.py --recipe fsdp --steps 6 --warmup 2" \
    "200:old_pipe_$rep:python -u bench.py --recipe pipe --steps 6 --warmup 2" "200:old_ppd_$rep:python -u bench.py --recipe pipe_ddp --steps 6 --warmup 2" || exit $?
  DPC_GEMM_TABLE_PATH=$DPC_GEMM_TUNE_OUT scripts/gpu_step.sh "150:new_ddp_$rep:python -u bench.py" "200:new_fsdp_$rep:python -u bench.py --recipe fsdp --steps 6 --warmup 2" \
    "200:new_pipe_$rep:python -u bench.py --recipe pipe --steps 6 --warmup 2" "200:new_ppd_$rep:python -u bench.py --recipe pipe_ddp --steps 6 --warmup 2" || exit $?
done
scripts/gpu_step.sh "300:off_break:python -u bench/offload.py --breakdown"
