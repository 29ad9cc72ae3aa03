#!/bin/bash
# round 5 job 33: GPU kernel/model tests with the GEMM store policy 15 default; attention output
# store policy A/B (DPC_ATTN_SPOL 0 / 1 / 2, interleaved); DDP bench new vs the round-start tree
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_fp32_gpu.py tests/test_model_gpu.py -m gpu > gpurun_out/r5_t33.log 2>&1 \
  || { tail -30 gpurun_out/r5_t33.log; exit 1; }
tail -2 gpurun_out/r5_t33.log
for r in 1 2 3; do
  for sp in 0 1 2; do
    echo "== DPC_ATTN_SPOL=$sp"
    DPC_ATTN_SPOL=$sp timeout -k 10 100 python -u bench/attn_time.py || exit $?
  done
done > gpurun_out/r5_attn_pol.log 2>&1
grep -v amdgpu.ids gpurun_out/r5_attn_pol.log
for r in 1 2; do
  echo "== new"; timeout -k 10 200 python -u bench.py || exit $?
  echo "== old"; (cd ab_old && timeout -k 10 200 python -u bench.py) || exit $?
done > gpurun_out/r5_bench33.log 2>&1
grep -v amdgpu.ids gpurun_out/r5_bench33.log | cut -c1-160
