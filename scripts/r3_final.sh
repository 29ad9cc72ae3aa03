#!/bin/bash
# End-of-session check (round 3): the driver's GPU tiers + the four recipe benches, then a
# rocprofv3 kernel table and per-step busy / idle table for each recipe.
bash scripts/round_check.sh || exit $?
for r in ddp fsdp pipe pipe_ddp; do
  bash scripts/prof_bench.sh r3_$r --recipe $r || exit $?
done
