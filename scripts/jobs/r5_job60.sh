#!/bin/bash
# round 5 job 60: final DDP step trace (kernel table, per-dispatch sequence)
mkdir -p gpurun_out
scripts/prof_bench.sh r5s60 || exit $?
