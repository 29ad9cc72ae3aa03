#!/bin/bash
# round 6 job 10: attn_fwd3_kernel (var 9) as the hd-64 forward default with its rescale update in
# asm: every GPU test + smoke, forward timing against fwd2 (var 6), DDP A/B against the round-start
# tree, step kernel table
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_step.sh "600:r6_gputests10:python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "120:r6_smoke10:python -u __graft_entry__.py" || exit $?
grep -q " passed" gpurun_out/r6_gputests10.log && ! grep -q "FAILED" gpurun_out/r6_gputests10.log || echo "=== GPU TESTS FAILED (continuing)"
for r in 1 2 3; do
  for v in 6 9; do
    echo -n "var $v: "; DPC_ATTN_VAR=$v,1 timeout -k 10 120 python -u bench/attn_time.py --rounds 5 --iters 10 2>/dev/null \
      | grep '^{' || exit 4
  done
done | tee gpurun_out/r6_attn10_var.log || exit 4
for r in 1 2; do
  echo "== new"; timeout -k 10 200 python -u bench.py || exit $?
  echo "== old"; (cd ab_old && timeout -k 10 200 python -u bench.py) || exit $?
done > gpurun_out/r6_bench10.log 2>&1
grep -v amdgpu.ids gpurun_out/r6_bench10.log | sed 's/"unit".*//'
scripts/prof_bench.sh r6s10 || exit $?
