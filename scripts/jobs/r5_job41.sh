#!/bin/bash
# round 5 job 41: branch-free embedding backward loads; the whole GPU suite on the current tree
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > gpurun_out/r5_t41.log 2>&1 \
  || { tail -30 gpurun_out/r5_t41.log; exit 1; }
tail -2 gpurun_out/r5_t41.log
timeout -k 10 200 python -u bench/emb_bwd_time.py 2>&1 | grep -v amdgpu.ids || exit 1
(cd ab_old && timeout -k 10 200 python -u bench/emb_bwd_time.py 2>&1 | grep -v amdgpu.ids) || true
