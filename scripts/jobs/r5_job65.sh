#!/bin/bash
# round 5 job 65: forward variants 6 / 7 (persistent) and the separate delta pre-pass, on the final tree
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "6,1 0" "7,1 0" "6,1 1"; do
    set -- $cfg
    echo "== VAR=$1 PRE=$2"; DPC_ATTN_VAR=$1 DPC_ATTN_PRE=$2 timeout -k 10 100 python -u bench/attn_time.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
