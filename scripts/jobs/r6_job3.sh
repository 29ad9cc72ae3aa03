#!/bin/bash
# round 6 job 3: the FFN down projection's residual add / act / dropout moved into the next
# layer's LN1 (plain bias GEMM for z2): LN / GEMM / model GPU tests, DDP A/B against the round-start
# tree, the other recipes, the step's kernel table; then the stock PyTorch yardsticks
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
(while sleep 45; do date >> gpurun_out/r6_hb.txt; done) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "layernorm or aux_deriv or act_grad_epilogue or v9_forward or decode or model or recipe or gpt2 or graph or kv" \
  > gpurun_out/r6j3_tests.log 2>&1 || { tail -30 gpurun_out/r6j3_tests.log; exit 3; }
tail -2 gpurun_out/r6j3_tests.log
for r in 1 2; do
  echo "== new"; timeout -k 10 200 python -u bench.py || exit $?
  echo "== old"; (cd ab_old && timeout -k 10 200 python -u bench.py) || exit $?
done > gpurun_out/r6_bench3.log 2>&1
grep -v amdgpu.ids gpurun_out/r6_bench3.log | sed 's/"unit".*//'
scripts/prof_bench.sh r6s3 || exit $?
for rc in fsdp pipe pipe_ddp; do
  timeout -k 10 300 python -u bench.py --recipe $rc --steps 6 --warmup 2 > gpurun_out/r6_b_$rc.log 2>&1 || exit $?
  grep '^{' gpurun_out/r6_b_$rc.log | cut -c1-170
done
