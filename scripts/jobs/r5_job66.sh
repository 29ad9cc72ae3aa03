#!/bin/bash
# round 5 job 66: the act' input-gradient product (EPI 8) alone under impl 22 / 20 / 16 instead of
# the table's 25, in the step (one table key changed per arm)
mkdir -p gpurun_out
for r in 1 2; do
  for t in base 22 20 16; do
    if [ $t = base ]; then unset DPC_GEMM_TABLE_PATH; else export DPC_GEMM_TABLE_PATH=bench/_tab_epi8_$t.json; fi
    echo "== table $t"; timeout -k 10 200 python -u bench.py 2>&1 | grep -v amdgpu.ids | grep -o '"value": [0-9.]*' || exit 1
  done
done
