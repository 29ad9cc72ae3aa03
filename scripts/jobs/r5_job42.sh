#!/bin/bash
# round 5 job 42: embedding backward with run-length groups, against the committed tree (ab_head,
# a built worktree of HEAD), interleaved; the embedding GPU tests first
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "emb" > gpurun_out/r5_t42.log 2>&1 || { tail -30 gpurun_out/r5_t42.log; exit 1; }
tail -1 gpurun_out/r5_t42.log
for r in 1 2 3; do
  echo "== new"; timeout -k 10 100 python -u bench/emb_bwd_time.py 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== head"; (cd ab_head && timeout -k 10 100 python -u bench/emb_bwd_time.py 2>&1 | grep -v amdgpu.ids) || exit 1
done
