#!/bin/bash
# Row-coalesced v7 plain epilogue (this tree) vs HEAD (ab_old/, full tree copy built from HEAD):
# GEMM numerics, then GEMM A/B on the GPT-2 small / XL products and DDP / FSDP benches, alternating.
R=$PWD
scripts/gpu_step.sh "300:t_gemm:python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_table_gpu.py -x -q --timeout 120 --timeout-method thread -k 'gemm or table'" || exit $?
for rep in 1 2; do
  for v in old new; do
    d=$R; [ $v = old ] && d=$R/ab_old
    (cd $d && timeout -k 10 200 python -u bench/gemm_ab.py --shapes gpt2s --impls 20 19 --rounds 3 --iters 5 > $R/gpurun_out/co_gemm_${v}_$rep.log 2>&1) || exit $?
    (cd $d && timeout -k 10 150 python -u bench.py > $R/gpurun_out/co_ddp_${v}_$rep.log 2>&1) || exit $?
    echo "$v $rep ddp: $(grep -o '"value": [0-9.]*' $R/gpurun_out/co_ddp_${v}_$rep.log)"
  done
done
for v in old new; do
  d=$R; [ $v = old ] && d=$R/ab_old
  (cd $d && timeout -k 10 200 python -u bench.py --recipe fsdp --steps 6 --warmup 2 > $R/gpurun_out/co_fsdp_${v}.log 2>&1) || exit $?
  echo "$v fsdp: $(grep -o '"value": [0-9.]*' $R/gpurun_out/co_fsdp_${v}.log)"
done
