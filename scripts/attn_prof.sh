#!/bin/bash
# Per-kernel times of the attention kernels (GPT-2 small shape, B=64 S=1023 H=12) at hd 64 / 32.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for hd in ${HDS:-64 32}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/attnprof_$hd -o run -- \
    python3 $R/bench/attn_one.py --N 64 --S 1023 --H 12 --hd $hd --iters 10 --bwd || exit $?
  python3 $R/scripts/kstats.py $R/gpurun_out/attnprof_$hd/run_results.db "attention hd=$hd B=64 S=1023 H=12" --top 8
done
