#!/bin/bash
# round 6 job 44 (final tree, relinked library): every GPU test + smoke + the default bench
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_step.sh "700:r6_gputests44:python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread" \
  "120:r6_smoke44:python -u __graft_entry__.py" \
  "200:b44_ddp:python -u bench.py" || exit $?
grep -q " passed" gpurun_out/r6_gputests44.log && ! grep -q "FAILED" gpurun_out/r6_gputests44.log || echo "=== GPU TESTS FAILED"
