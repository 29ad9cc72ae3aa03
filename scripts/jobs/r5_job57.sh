#!/bin/bash
# round 5 job 57: backward variant sweep again under the heaviest-first block order
mkdir -p gpurun_out
for r in 1 2; do
  for v in "6,1" "6,0" "6,2" "6,3"; do
    echo "== DPC_ATTN_VAR=$v"; DPC_ATTN_VAR=$v timeout -k 10 100 python -u bench/attn_time.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
