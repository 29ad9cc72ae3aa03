#!/bin/bash
# Kernel trace of a short bench.py run + per-step busy/idle breakdown:
#   scripts/prof_bench.sh <tag> [bench args...]
set -e
R=$GRAFT_REPO_ROOT
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$tag -o b -- \
  python3 $R/bench.py --steps 10 --warmup 3 "$@" > $R/gpurun_out/prof_$tag.log 2>&1
cd $R
db=$(ls gpurun_out/prof_$tag/*/b_results.db 2>/dev/null | head -1 || true)
[ -z "$db" ] && db=$(find gpurun_out/prof_$tag -name "*.db" | head -1)
python3 scripts/step_gaps.py $db --steps 8 --seq gpurun_out/prof_${tag}_seq.txt > gpurun_out/prof_${tag}_steps.md
python3 scripts/kstats.py $db "bench $tag" > gpurun_out/prof_${tag}_kstats.md
tail -3 gpurun_out/prof_$tag.log
head -12 gpurun_out/prof_${tag}_steps.md
# the trace databases are large (gpurun copies back at most 64 MiB): keep the summaries
[ -n "$KEEP_DB" ] || rm -rf gpurun_out/prof_$tag
