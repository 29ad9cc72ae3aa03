#!/bin/bash
# round 5 job 37: DDP step trace with the branch-free LayerNorm backward (prefetch on)
mkdir -p gpurun_out
scripts/prof_bench.sh r5s37 || exit $?
grep -E "ln_bwd|ln_fwd" gpurun_out/prof_r5s37_kstats.md
grep ln_bwd gpurun_out/prof_r5s37_seq.txt | awk '{print $1}' | tr '\n' ' '
