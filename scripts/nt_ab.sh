#!/bin/bash
# Non-temporal v7 epilogue stores (this tree) vs the HEAD kernels (ab_old/, a full tree copy
# built from HEAD): GEMM A/B on the GPT-2 small / XL products, DDP and FSDP benches, alternating.
R=$PWD
for rep in 1 2; do
  for v in old new; do
    d=$R; [ $v = old ] && d=$R/ab_old
    (cd $d && timeout -k 10 200 python -u bench/gemm_ab.py --shapes gpt2s --impls 20 19 --rounds 3 --iters 5 > $R/gpurun_out/nt_gemm_${v}_$rep.log 2>&1) || exit $?
    (cd $d && timeout -k 10 150 python -u bench.py > $R/gpurun_out/nt_ddp_${v}_$rep.log 2>&1) || exit $?
    echo "$v $rep ddp: $(grep -o '"value": [0-9.]*' $R/gpurun_out/nt_ddp_${v}_$rep.log)"
  done
done
for v in old new; do
  d=$R; [ $v = old ] && d=$R/ab_old
  (cd $d && timeout -k 10 200 python -u bench.py --recipe fsdp --steps 6 --warmup 2 > $R/gpurun_out/nt_fsdp_${v}.log 2>&1) || exit $?
  echo "$v fsdp: $(grep -o '"value": [0-9.]*' $R/gpurun_out/nt_fsdp_${v}.log)"
done
