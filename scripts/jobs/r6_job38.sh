#!/bin/bash
# round 6 job 38: the weight-gradient products of the GPT-2 small step (K = 64 x 1023 tokens)
# swept over forced split-K counts against the planner's choice (s0), table path (-1) and v7
# sched 6 (25, the step's kernel)
mkdir -p gpurun_out
timeout -k 10 400 python -u bench/wgrad_splits.py --T 65472 --impls -1 25 \
  --splits 0 1 2 3 4 5 6 7 8 10 12 16 > gpurun_out/r6_wgrad_splits.log 2>&1
rc=$?; cat gpurun_out/r6_wgrad_splits.log | grep -v amdgpu.ids; exit $rc
