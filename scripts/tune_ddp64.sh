#!/bin/bash
# Extend the GEMM table with the DDP bench shapes at B=64, then A/B it and profile the step.
export DPC_GEMM_TUNE_OUT=gpurun_out/gemm_tuned.json
cp distributed_pytorch_cookbook_amd/ops/gemm_tuned.json gpurun_out/gemm_tuned.json
scripts/gpu_step.sh "200:tune64:DPC_GEMM_TUNE=1 python -u bench.py --steps 3 --warmup 2" \
  "150:ab64_0:DPC_GEMM_TABLE=0 python -u bench.py" \
  "150:ab64_1:DPC_GEMM_TUNE=1 python -u bench.py" \
  "300:prof:scripts/prof_bench.sh v15"
