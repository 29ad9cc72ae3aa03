#!/bin/bash
# PMC counters for one GEMM shape and impl, one counter group per rocprofv3 pass:
#   scripts/pmc_gemm.sh <tag> <impl> <M> <N> <K> <layout>
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=$1; impl=$2; M=$3; N=$4; K=$5; lay=$6
run() {  # $1 = pass name, rest = counters
  local pass=$1; shift
  timeout -k 5 60 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmc_${tag}_${pass} -o p -- \
    python3 $R/bench/gemm_one.py --M $M --N $N --K $K --layout $lay --impl $impl --iters 5
}
run a SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA
run b SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS
run c TCC_HIT_sum TCC_MISS_sum
