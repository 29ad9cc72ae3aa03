#!/bin/bash
# round 5 job 38: every plain GEMM of the DDP step, ours vs hipBLASLt (torch.mm)
mkdir -p gpurun_out
timeout -k 10 400 python -u bench/step_gemms_vs_blas.py > gpurun_out/r5_gemm_blas.log 2>&1 || { tail -20 gpurun_out/r5_gemm_blas.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5_gemm_blas.log
