#!/bin/bash
# round 6 job 17: validation of the tree after the IPC work: every GPU test + smoke, then the DDP
# bench against the round-start tree (same box) and the step kernel table
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_step.sh "600:r6_gputests17:python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread" \
  "120:r6_smoke17:python -u __graft_entry__.py" || exit $?
grep -q " passed" gpurun_out/r6_gputests17.log && ! grep -q "FAILED" gpurun_out/r6_gputests17.log || echo "=== GPU TESTS FAILED (continuing)"
for r in 1 2; do
  echo "== new"; timeout -k 10 200 python -u bench.py || exit $?
  echo "== old"; (cd ab_old && timeout -k 10 200 python -u bench.py) || exit $?
done > gpurun_out/r6_bench17.log 2>&1
grep -v amdgpu.ids gpurun_out/r6_bench17.log | sed 's/"unit".*//'
scripts/prof_bench.sh r6s17 || exit $?
