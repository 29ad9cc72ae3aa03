#!/bin/bash
# round 6 job 46 (final tree after the dQ experiments, library rebuilt from the same sources): every GPU test + smoke + the default bench
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_step.sh "700:r6_gputests46:python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread" \
  "120:r6_smoke46:python -u __graft_entry__.py" \
  "200:b46_ddp:python -u bench.py" || exit $?
grep -q " passed" gpurun_out/r6_gputests46.log && ! grep -q "FAILED" gpurun_out/r6_gputests46.log || echo "=== GPU TESTS FAILED"
