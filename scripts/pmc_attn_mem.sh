#!/bin/bash
# HBM / L2 traffic of the attention forward variants: FETCH_SIZE, TCC hit / miss.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in ${VARS:-0 6}; do
  for pass in "f:FETCH_SIZE" "h:TCC_HIT_sum TCC_MISS_sum" "w:SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES"; do
    tag=${pass%%:*}; cnt=${pass#*:}
    DPC_ATTN_VAR=$v,1 timeout -s KILL 60 rocprofv3 --pmc $cnt -d $R/gpurun_out/pmcm_${v}_$tag -o p -- \
      python3 $R/bench/attn_one.py --N 64 --S 1023 --H 12 --iters 3 > /dev/null 2>&1 || exit 1
    echo "== var $v pass $tag"
    python3 $R/scripts/pmc_summary.py $(find $R/gpurun_out/pmcm_${v}_$tag -name "*.db" | head -1) attn_fwd
    rm -rf $R/gpurun_out/pmcm_${v}_$tag
  done
done
