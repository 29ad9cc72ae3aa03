#!/bin/bash
# round 5 job 69: the whole GPU suite with the f32-plain store default (77), then 77 vs 15 again on
# another box, interleaved
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/r5_t69.log 2>&1 \
  || { tail -30 gpurun_out/r5_t69.log; exit 1; }
tail -1 gpurun_out/r5_t69.log
for r in 1 2 3; do
  for nt in 77 15; do
    echo "== NT $nt"; DPC_GEMM_NT=$nt timeout -k 10 200 python -u bench.py 2>&1 | grep -v amdgpu.ids | grep -o '"value": [0-9.]*' || exit 1
  done
done
