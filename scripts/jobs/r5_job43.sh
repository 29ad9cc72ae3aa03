#!/bin/bash
# round 5 job 43: LayerNorm forward with every row load issued up front; LN tests, then the
# forward / backward cases against the committed tree (ab_head), interleaved
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu \
  > gpurun_out/r5_t43.log 2>&1 || { tail -30 gpurun_out/r5_t43.log; exit 1; }
tail -1 gpurun_out/r5_t43.log
for r in 1 2; do
  echo "== new"; timeout -k 10 100 python -u bench/ln_bwd_ab.py --rounds 2 2>&1 | grep -v amdgpu.ids | grep "fwd\|\"pf\": 1" || exit 1
  echo "== head"; (cd ab_head && timeout -k 10 100 python -u bench/ln_bwd_ab.py --rounds 2 2>&1 | grep -v amdgpu.ids | grep "fwd\|\"pf\": 1") || exit 1
done
