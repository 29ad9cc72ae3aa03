#!/bin/bash
# Re-measure the whole GEMM table from scratch (every candidate impl) over the four bench
# recipes at their default batches -> gpurun_out/gemm_tuned_full.json; then A/B old vs new.
export DPC_GEMM_TUNE_OUT=gpurun_out/gemm_tuned_full.json
rm -f gpurun_out/gemm_tuned_full.json
DPC_GEMM_TABLE=0 DPC_GEMM_TUNE=1 scripts/gpu_step.sh "200:rt_ddp:python -u bench.py --steps 2 --warmup 2" \
  "300:rt_fsdp:python -u bench.py --recipe fsdp --steps 2 --warmup 2" \
  "300:rt_pipe:python -u bench.py --recipe pipe --steps 2 --warmup 2" \
  "300:rt_ppd:python -u bench.py --recipe pipe_ddp --steps 2 --warmup 2" || exit $?
scripts/gpu_step.sh "150:old_ddp:python -u bench.py" "200:old_fsdp:python -u bench.py --recipe fsdp --steps 6 --warmup 2" || exit $?
cp gpurun_out/gemm_tuned_full.json distributed_pytorch_cookbook_amd/ops/gemm_tuned.json
scripts/gpu_step.sh "150:new_ddp:python -u bench.py" "200:new_fsdp:python -u bench.py --recipe fsdp --steps 6 --warmup 2" \
  "200:new_pipe:python -u bench.py --recipe pipe --steps 6 --warmup 2" "200:new_ppd:python -u bench.py --recipe pipe_ddp --steps 6 --warmup 2"
