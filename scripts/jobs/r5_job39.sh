#!/bin/bash
# round 5 job 39: row-chunked LM head + CE (logits re-read from the Infinity Cache) at today's
# kernels, with the default (sc0 sc1 nt) and plain GEMM output stores
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "0 15" "2560 15" "2560 3" "4096 15" "4096 3" "8192 15"; do
    set -- $cfg
    echo "== chunk=$1 nt=$2"
    DPC_HEAD_CHUNK=$1 DPC_GEMM_NT=$2 timeout -k 10 200 python -u bench.py || exit $?
  done
done > gpurun_out/r5_chunk39.log 2>&1
grep -v amdgpu.ids gpurun_out/r5_chunk39.log | sed 's/"unit".*//'
