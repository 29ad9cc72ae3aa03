#!/bin/bash
# round 6 job 8 (job 6 again, tests without -x): every layer (the last one included) hands its FFN output to the next LayerNorm
# (the final norm, or a materialising pass at a pipeline boundary): all GPU tests, DDP A/B against
# the round-start tree, the step's kernel table
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_step.sh "600:r6_gputests8:python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "120:r6_smoke8:python -u __graft_entry__.py" || exit $?
grep -q " passed" gpurun_out/r6_gputests8.log && ! grep -q "FAILED" gpurun_out/r6_gputests8.log || echo "=== GPU TESTS FAILED (continuing)"
for r in 1 2; do
  echo "== new"; timeout -k 10 200 python -u bench.py || exit $?
  echo "== old"; (cd ab_old && timeout -k 10 200 python -u bench.py) || exit $?
done > gpurun_out/r6_bench8.log 2>&1
grep -v amdgpu.ids gpurun_out/r6_bench8.log | sed 's/"unit".*//'
scripts/prof_bench.sh r6s8 || exit $?
for v in 9 10; do
  DPC_ATTN_VAR=$v,1 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 \
    --timeout-method thread -k "attention_fwd_bwd or attention_long" > gpurun_out/r6_attn_t$v.log 2>&1 \
    || { tail -20 gpurun_out/r6_attn_t$v.log; exit 5; }
  tail -1 gpurun_out/r6_attn_t$v.log
done
for r in 1 2 3; do
  for v in 6 9 5 10; do
    echo -n "var $v: "; DPC_ATTN_VAR=$v,1 timeout -k 10 120 python -u bench/attn_time.py --rounds 5 --iters 10 2>/dev/null \
      | grep '^{' || exit 4
  done
done | tee gpurun_out/r6_attn_var.log
