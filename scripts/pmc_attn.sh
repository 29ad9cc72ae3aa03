#!/bin/bash
# PMC counters for the attention kernels: scripts/pmc_attn.sh <tag> [--bwd]
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=$1; shift
run() {
  local pass=$1; shift
  timeout -k 5 60 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmc_${tag}_${pass} -o p -- \
    python3 $R/bench/attn_one.py --N 64 --S 1023 --H 12 --iters 3 $EXTRA
}
EXTRA="$*"
run a SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA
run b SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS
run c SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_SCA
