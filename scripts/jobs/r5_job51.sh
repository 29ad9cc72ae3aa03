#!/bin/bash
# round 5 job 51: forward O rescale as an unconditional packed multiply (no join copies):
# attention tests, then attn_time against ab_head, interleaved
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "attn or attention" > gpurun_out/r5_t51.log 2>&1 || { tail -30 gpurun_out/r5_t51.log; exit 1; }
tail -1 gpurun_out/r5_t51.log
for r in 1 2 3; do
  echo "== new"; timeout -k 10 100 python -u bench/attn_time.py 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== head"; (cd ab_head && timeout -k 10 100 python -u bench/attn_time.py 2>&1 | grep -v amdgpu.ids) || exit 1
done
