#!/bin/bash
# round 5 job 45: attention scalar-instruction trim (no M0 save / restore, item offsets formed
# once per item, 32-bit descriptor math): attention tests, then the A/B against ab_head
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp32_gpu.py -m gpu \
  -k "attn or attention" > gpurun_out/r5_t45.log 2>&1 || { tail -30 gpurun_out/r5_t45.log; exit 1; }
tail -1 gpurun_out/r5_t45.log
for r in 1 2 3; do
  echo "== new"; timeout -k 10 100 python -u bench/attn_time.py 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== head"; (cd ab_head && timeout -k 10 100 python -u bench/attn_time.py 2>&1 | grep -v amdgpu.ids) || exit 1
done
