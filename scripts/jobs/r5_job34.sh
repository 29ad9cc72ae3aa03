#!/bin/bash
# round 5 job 34: DDP step kernel trace with the per-dispatch sequence of one step
mkdir -p gpurun_out
scripts/prof_bench.sh r5s34 || exit $?
head -5 gpurun_out/prof_r5s34_seq.txt
