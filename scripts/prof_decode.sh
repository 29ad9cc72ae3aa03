#!/bin/bash
# Kernel statistics of bench/generate.py (greedy decode variants) on one MI355X.
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_decode -o d -- \
  python3 $R/bench/generate.py "$@" > $R/gpurun_out/prof_decode.log 2>&1
cd $R
db=$(find gpurun_out/prof_decode -name "*.db" | head -1)
python3 scripts/kstats.py $db "decode $*" > gpurun_out/prof_decode_kstats.md
head -40 gpurun_out/prof_decode_kstats.md
