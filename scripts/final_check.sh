#!/bin/bash
# End-of-session check: the driver's GPU tiers + the four recipe benches at their defaults, then a
# rocprofv3 kernel table and per-step busy/idle table for each recipe.
bash scripts/round_check.sh || exit $?
for r in ddp fsdp pipe pipe_ddp; do
  bash scripts/prof_bench.sh s4_$r --recipe $r || exit $?
done
