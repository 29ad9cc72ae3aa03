#!/bin/bash
# round 5 job 53: the whole GPU suite after removing the attention store-policy switch and
# parametrizing the LayerNorm test over the backward prefetch
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/r5_t53.log 2>&1 \
  || { tail -30 gpurun_out/r5_t53.log; exit 1; }
tail -2 gpurun_out/r5_t53.log
timeout -k 10 100 python -u bench/attn_time.py 2>&1 | grep -v amdgpu.ids
