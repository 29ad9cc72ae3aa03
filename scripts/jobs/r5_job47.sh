#!/bin/bash
# round 5 job 47: GEMM descriptor clamp as a scalar select (prep()): GEMM tests, the plain step
# GEMMs and the fused FFN decomposition against the committed tree (ab_head), then the DDP bench A/B
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "gemm" > gpurun_out/r5_t47.log 2>&1 || { tail -30 gpurun_out/r5_t47.log; exit 1; }
tail -1 gpurun_out/r5_t47.log
for r in 1 2; do
  echo "== new"; timeout -k 10 150 python -u bench/epi_decomp.py --rounds 2 --iters 10 --only up_plain up_full dg_plain dg_full dn_full 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== head"; (cd ab_head && timeout -k 10 150 python -u bench/epi_decomp.py --rounds 2 --iters 10 --only up_plain up_full dg_plain dg_full dn_full 2>&1 | grep -v amdgpu.ids) || exit 1
done
for r in 1 2; do
  echo "== bench new"; timeout -k 10 200 python -u bench.py 2>&1 | grep -v amdgpu.ids | sed 's/"unit".*//' || exit 1
  echo "== bench head"; (cd ab_head && timeout -k 10 200 python -u bench.py 2>&1 | grep -v amdgpu.ids | sed 's/"unit".*//') || exit 1
done
