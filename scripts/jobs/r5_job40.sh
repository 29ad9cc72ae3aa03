#!/bin/bash
# round 5 job 40: attention backward variants on today's kernels (DPC_ATTN_VAR fwd,bwd), interleaved
mkdir -p gpurun_out
for r in 1 2; do
  for v in "6,1" "6,0" "6,2" "6,3" "5,1" "8,1"; do
    echo "== DPC_ATTN_VAR=$v"
    DPC_ATTN_VAR=$v timeout -k 10 100 python -u bench/attn_time.py || exit $?
  done
done > gpurun_out/r5_attn_var40.log 2>&1
grep -v amdgpu.ids gpurun_out/r5_attn_var40.log
