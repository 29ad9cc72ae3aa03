#!/bin/bash
# round 6 job 27: kernel table of the reference CLI default model after the f32 LM-head dgrad
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/prof_bench.sh r6ref2 --model ref --seq_len 256 --batch_size 64 || exit $?
head -30 gpurun_out/prof_r6ref2_kstats.md
