#!/bin/bash
# round 5 job 59: LayerNorm backward grid in the step (DPC_LN_BWD_BLOCKS 256 / 384 / default)
mkdir -p gpurun_out
for r in 1 2; do
  for nb in 0 256 384; do
    echo "== blocks $nb"; DPC_LN_BWD_BLOCKS=$nb timeout -k 10 200 python -u bench.py 2>&1 | grep -v amdgpu.ids | sed 's/"unit".*//' || exit 1
  done
done
