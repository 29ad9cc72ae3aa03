#!/bin/bash
# round 5 job 35: is the LayerNorm backward's 154 -> 207 us a side effect of the GEMM store policy
# (sc0 sc1 nt outputs bypassing the caches its dy read hit)?  DDP step traces at policy 3 and 15
mkdir -p gpurun_out
DPC_GEMM_NT=3 scripts/prof_bench.sh r5p3 || exit $?
DPC_GEMM_NT=15 scripts/prof_bench.sh r5p15 || exit $?
for t in r5p3 r5p15; do echo "== $t"; head -22 gpurun_out/prof_${t}_steps.md | tail -12; done
