#!/bin/bash
# forward GELU epilogues (gemm3 epi_tile, v8) in packed-f32 math (this tree) vs scalar (ab_old/, a
# tree copy of HEAD): GEMM numerics, the fused forward GELU products, then the DDP / FSDP benches.
R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_table_gpu.py -x -q --timeout 120 --timeout-method thread -k 'gemm or table' > gpurun_out/t_gemm.log 2>&1 || { tail -30 gpurun_out/t_gemm.log; exit 1; }; tail -3 gpurun_out/t_gemm.log
for rep in 1 2; do
  for v in old new; do
    d=$R; [ $v = old ] && d=$R/ab_old
    (cd $d && timeout -k 10 200 python -u bench/gemm_ab.py --shapes fused --only s_up_fwd s_down_fwd xl_up_fwd xl_down_fwd --impls 20 --rounds 3 --iters 5 > $R/gpurun_out/pf_fw_gemm_${v}_$rep.log 2>&1) || exit $?
    (cd $d && timeout -k 10 150 python -u bench.py > $R/gpurun_out/pf_fw_ddp_${v}_$rep.log 2>&1) || exit $?
    echo "$v $rep ddp: $(grep -o '"value": [0-9.]*' $R/gpurun_out/pf_fw_ddp_${v}_$rep.log)"
  done
done
for v in old new; do
  d=$R; [ $v = old ] && d=$R/ab_old
  (cd $d && timeout -k 10 200 python -u bench.py --recipe fsdp --steps 6 --warmup 2 > $R/gpurun_out/pf_fw_fsdp_${v}.log 2>&1) || exit $?
  echo "$v fsdp: $(grep -o '"value": [0-9.]*' $R/gpurun_out/pf_fw_fsdp_${v}.log)"
done
