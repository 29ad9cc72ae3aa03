#!/bin/bash
# round 5 job 10: attention variant sweep after the dK / dV VALU cuts (DPC_ATTN_VAR=<fwd>,<bwd>)
mkdir -p gpurun_out
for v in 6,1 5,1 6,0 6,3 7,1 8,1 6,2 6,1; do
  echo "== var $v"
  DPC_ATTN_VAR=$v timeout -k 10 120 python -u bench/attn_time.py || exit $?
done > gpurun_out/r5_attn_var.log 2>&1
cat gpurun_out/r5_attn_var.log
