#!/bin/bash
# round 5 job 55: attention backward block order (DPC_ATTN_ORDER=1: heaviest causal blocks first over
# the whole grid): attention tests under it, attn_time and the DDP bench, interleaved with order 0
mkdir -p gpurun_out
DPC_ATTN_ORDER=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "attn or attention" > gpurun_out/r5_t55.log 2>&1 || { tail -30 gpurun_out/r5_t55.log; exit 1; }
tail -1 gpurun_out/r5_t55.log
for r in 1 2 3; do
  for o in 0 1; do
    echo "== order $o"; DPC_ATTN_ORDER=$o timeout -k 10 100 python -u bench/attn_time.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
for r in 1 2; do
  for o in 0 1; do
    echo "== bench order $o"; DPC_ATTN_ORDER=$o timeout -k 10 200 python -u bench.py 2>&1 | grep -v amdgpu.ids | sed 's/"unit".*//' || exit 1
  done
done
