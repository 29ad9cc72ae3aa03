#!/bin/bash
# round 6 job 42 (final tree, after the IPC stream fix): every GPU test + smoke, the four recipes, the DDP kernel table
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_step.sh "700:r6_gputests42:python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread" \
  "120:r6_smoke42:python -u __graft_entry__.py" \
  "200:b42_ddp:python -u bench.py" \
  "200:b42_fsdp:python -u bench.py --recipe fsdp --steps 8 --warmup 3" \
  "200:b42_pipe:python -u bench.py --recipe pipe --steps 8 --warmup 3" \
  "200:b42_ppd:python -u bench.py --recipe pipe_ddp --steps 8 --warmup 3" || exit $?
grep -q " passed" gpurun_out/r6_gputests42.log && ! grep -q "FAILED" gpurun_out/r6_gputests42.log || echo "=== GPU TESTS FAILED"
scripts/prof_bench.sh r6s42 || exit $?
