#!/bin/bash
# one PMC pass (instruction counts) over bench/attn_one.py: scripts/pmc_attn_c.sh <tag>
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 5 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
  -d $R/gpurun_out/pmc_$1_c -o p -- python3 $R/bench/attn_one.py --N 64 --S 1023 --H 12 --iters 3
