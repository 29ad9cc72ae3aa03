#!/bin/bash
# round 6 job 47 (final tree, library from a full __graft_entry__.build()): every GPU test + smoke + the default bench
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_step.sh "700:r6_gputests47:python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread" \
  "120:r6_smoke47:python -u __graft_entry__.py" \
  "200:b47_ddp:python -u bench.py" || exit $?
grep -q " passed" gpurun_out/r6_gputests47.log && ! grep -q "FAILED" gpurun_out/r6_gputests47.log || echo "=== GPU TESTS FAILED"
