#!/bin/bash
# This tree vs ab_old/ (the tree before the act' prefetch and the packed-f32 GELU / GELU'
# epilogues), alternating on one box: DDP, FSDP and PP x DP benches.
R=$PWD
for rep in 1 2; do
  for v in old new; do
    d=$R; [ $v = old ] && d=$R/ab_old
    (cd $d && timeout -k 10 150 python -u bench.py > $R/gpurun_out/all_ddp_${v}_$rep.log 2>&1) || exit $?
    (cd $d && timeout -k 10 200 python -u bench.py --recipe fsdp --steps 6 --warmup 2 > $R/gpurun_out/all_fsdp_${v}_$rep.log 2>&1) || exit $?
    (cd $d && timeout -k 10 200 python -u bench.py --recipe pipe_ddp --steps 6 --warmup 2 > $R/gpurun_out/all_ppd_${v}_$rep.log 2>&1) || exit $?
    echo "$v $rep ddp $(grep -o '"value": [0-9.]*' $R/gpurun_out/all_ddp_${v}_$rep.log) fsdp $(grep -o '"value": [0-9.]*' $R/gpurun_out/all_fsdp_${v}_$rep.log) ppd $(grep -o '"value": [0-9.]*' $R/gpurun_out/all_ppd_${v}_$rep.log)"
  done
done
