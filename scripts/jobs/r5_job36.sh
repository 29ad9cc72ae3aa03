#!/bin/bash
# round 5 job 36: LayerNorm backward with branch-free row loads (+ next-row prefetch variant):
# numerics, the isolated A/B, then the DDP bench against the round-start tree
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "layernorm or ln_" > gpurun_out/r5_t36.log 2>&1 || { tail -30 gpurun_out/r5_t36.log; exit 1; }
tail -1 gpurun_out/r5_t36.log
timeout -k 10 200 python -u bench/ln_bwd_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
for r in 1 2; do
  for pf in 1 0; do
    echo "== new pf=$pf"; DPC_LN_BWD_PF=$pf timeout -k 10 200 python -u bench.py || exit $?
  done
  echo "== old"; (cd ab_old && timeout -k 10 200 python -u bench.py) || exit $?
done > gpurun_out/r5_bench36.log 2>&1
grep -v amdgpu.ids gpurun_out/r5_bench36.log | cut -c1-150
