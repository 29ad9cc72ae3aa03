#!/bin/bash
# round 6 job 6: every layer (the last one included) hands its FFN output to the next LayerNorm
# (the final norm, or a materialising pass at a pipeline boundary): all GPU tests, DDP A/B against
# the round-start tree, the step's kernel table
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_step.sh "600:r6_gputests6:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "120:r6_smoke6:python -u __graft_entry__.py" || exit $?
grep -q " passed" gpurun_out/r6_gputests6.log && ! grep -q "FAILED" gpurun_out/r6_gputests6.log || exit 3
for r in 1 2; do
  echo "== new"; timeout -k 10 200 python -u bench.py || exit $?
  echo "== old"; (cd ab_old && timeout -k 10 200 python -u bench.py) || exit $?
done > gpurun_out/r6_bench6.log 2>&1
grep -v amdgpu.ids gpurun_out/r6_bench6.log | sed 's/"unit".*//'
scripts/prof_bench.sh r6s6 || exit $?
