#!/bin/bash
# round 5 job 46: DDP bench of the current tree against the round-start tree (ab_old), interleaved,
# then the step's kernel trace
mkdir -p gpurun_out
for r in 1 2 3; do
  echo "== new"; timeout -k 10 200 python -u bench.py || exit $?
  echo "== old"; (cd ab_old && timeout -k 10 200 python -u bench.py) || exit $?
done > gpurun_out/r5_bench46.log 2>&1
grep -v amdgpu.ids gpurun_out/r5_bench46.log | sed 's/"unit".*//'
scripts/prof_bench.sh r5s46 || exit $?
