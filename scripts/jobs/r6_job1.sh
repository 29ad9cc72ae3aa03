#!/bin/bash
# round 6 job 1: GELU' stored by the up-projection forward (aux_deriv) + ACT_MUL input gradient:
# GEMM numerics, model GPU tests, DDP bench against the round-start tree (ab_old) interleaved,
# then the step's kernel trace
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "aux_deriv or act_grad_epilogue or v9_forward or v7_v8_v9 or impls_with_epilogue or v7d" \
  > gpurun_out/r6j1_tests.log 2>&1 || { tail -30 gpurun_out/r6j1_tests.log; exit 3; }
tail -2 gpurun_out/r6j1_tests.log
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r6j1_model.log 2>&1 || { tail -30 gpurun_out/r6j1_model.log; exit 3; }
tail -2 gpurun_out/r6j1_model.log
for r in 1 2; do
  echo "== new"; timeout -k 10 200 python -u bench.py || exit $?
  echo "== old"; (cd ab_old && timeout -k 10 200 python -u bench.py) || exit $?
done > gpurun_out/r6_bench1.log 2>&1
grep -v amdgpu.ids gpurun_out/r6_bench1.log | sed 's/"unit".*//'
scripts/prof_bench.sh r6s1 || exit $?
