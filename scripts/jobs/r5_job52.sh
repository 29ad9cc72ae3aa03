#!/bin/bash
# round 5 job 52: kernel trace of the pipe (GPT-2 medium) recipe
mkdir -p gpurun_out
scripts/prof_bench.sh r5pipe --recipe pipe --steps 6 --warmup 2 || exit $?
head -30 gpurun_out/prof_r5pipe_steps.md
