#!/bin/bash
# round 5 job 50: which GEMM table signatures the DDP step looks up
mkdir -p gpurun_out
timeout -k 10 200 python -u bench/step_gemm_keys.py > gpurun_out/r5_keys.log 2>&1 || { tail -20 gpurun_out/r5_keys.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5_keys.log | cut -c1-200
