#!/bin/bash
# Measure the per-shape GEMM implementation table (ops/gemm_tuned.json) on one MI355X over
# the four bench recipes at their default batches; the merged table lands in
# gpurun_out/gemm_tuned.json (copy it into the package).
export DPC_GEMM_TUNE_OUT=gpurun_out/gemm_tuned.json
cp distributed_pytorch_cookbook_amd/ops/gemm_tuned.json gpurun_out/gemm_tuned.json
DPC_GEMM_TUNE=1 scripts/gpu_step.sh "200:t_ddp:python -u bench.py --steps 3 --warmup 2" \
  "300:t_fsdp:python -u bench.py --recipe fsdp --steps 3 --warmup 2" \
  "300:t_pipe:python -u bench.py --recipe pipe --steps 3 --warmup 2" \
  "300:t_ppd:python -u bench.py --recipe pipe_ddp --steps 3 --warmup 2" || exit $?
cp gpurun_out/gemm_tuned.json distributed_pytorch_cookbook_amd/ops/gemm_tuned.json
scripts/gpu_step.sh "150:b_ddp:python -u bench.py" \
  "200:b_fsdp:python -u bench.py --recipe fsdp --steps 8 --warmup 3" \
  "200:b_pipe:python -u bench.py --recipe pipe --steps 8 --warmup 3" \
  "200:b_ppd:python -u bench.py --recipe pipe_ddp --steps 8 --warmup 3"
