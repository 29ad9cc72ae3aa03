#!/bin/bash
# round 6 job 23 (final validation): every GPU test + smoke, DDP A/B against the round-start tree,
# the four recipes, the DDP step kernel table
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_step.sh "700:r6_gputests23:python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread" \
  "120:r6_smoke23:python -u __graft_entry__.py" || exit $?
grep -q " passed" gpurun_out/r6_gputests23.log && ! grep -q "FAILED" gpurun_out/r6_gputests23.log || echo "=== GPU TESTS FAILED (continuing)"
for r in 1 2; do
  echo "== new"; timeout -k 10 200 python -u bench.py || exit $?
  echo "== old"; (cd ab_old && timeout -k 10 200 python -u bench.py) || exit $?
done > gpurun_out/r6_bench23.log 2>&1
grep -v amdgpu.ids gpurun_out/r6_bench23.log | sed 's/"unit".*//'
scripts/gpu_step.sh "200:b23_fsdp:python -u bench.py --recipe fsdp --steps 8 --warmup 3" \
  "200:b23_pipe:python -u bench.py --recipe pipe --steps 8 --warmup 3" \
  "200:b23_ppd:python -u bench.py --recipe pipe_ddp --steps 8 --warmup 3" || exit $?
scripts/prof_bench.sh r6s23 || exit $?
