#!/bin/bash
# round 5 job 68: a separate store scope for the f32 GEMM outputs (residual stream, split-K slabs):
# DPC_GEMM_NT 15 (all sc0 sc1 nt) / 77 (f32 plain) / 109 (f32 sc1 nt), interleaved in the step
mkdir -p gpurun_out
DPC_GEMM_NT=77 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "gemm" > gpurun_out/r5_t68.log 2>&1 || { tail -30 gpurun_out/r5_t68.log; exit 1; }
tail -1 gpurun_out/r5_t68.log
for r in 1 2 3; do
  for nt in 15 77 109; do
    echo "== NT $nt"; DPC_GEMM_NT=$nt timeout -k 10 200 python -u bench.py 2>&1 | grep -v amdgpu.ids | grep -o '"value": [0-9.]*' || exit 1
  done
done
