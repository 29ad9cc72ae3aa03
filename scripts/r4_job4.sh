#!/bin/bash
# same-box A/B: e66e941 (ab_old/) vs this tree (scalar alpha, ER 4 default) vs this tree with the
# up-projection forward on v9 (bench/tables/gemm_tuned_g9fwd.json); FSDP old vs new; kernel
# profiles of the pipeline stage proxy (micro-batched vs one batch)
R=$PWD
scripts/gpu_step.sh "300:warm:python -u scripts/warm.py" || exit $?
(cd ab_old && timeout -k 10 300 python -u ../scripts/warm.py > $R/gpurun_out/warm_old.log 2>&1) || exit $?
for rep in 1 2 3; do
  (cd ab_old && timeout -k 10 150 python -u bench.py > $R/gpurun_out/e_old_$rep.log 2>&1) || exit $?
  timeout -k 10 150 python -u bench.py > gpurun_out/e_new_$rep.log 2>&1 || exit $?
  DPC_GEMM_TABLE_PATH=bench/tables/gemm_tuned_g9fwd.json timeout -k 10 150 python -u bench.py > gpurun_out/e_g9f_$rep.log 2>&1 || exit $?
  DPC_G9_ER=0 timeout -k 10 150 python -u bench.py > gpurun_out/e_er0_$rep.log 2>&1 || exit $?
done
for f in gpurun_out/e_*.log; do
  echo "$f $(grep -h '"value"' $f | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
(cd ab_old && timeout -k 10 200 python -u bench.py --recipe fsdp --steps 6 --warmup 2 > $R/gpurun_out/f_old.log 2>&1) || exit $?
DPC_GEMM_TABLE_PATH=bench/tables/gemm_tuned_g9fwd.json timeout -k 10 200 python -u bench.py --recipe fsdp --steps 6 --warmup 2 > gpurun_out/f_g9f.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --recipe fsdp --steps 6 --warmup 2 > gpurun_out/f_new.log 2>&1 || exit $?
for f in gpurun_out/f_*.log; do
  echo "$f $(grep -h '"value"' $f | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ppm -o run -- python -u bench/pp_stage_proxy.py --model gpt2-medium --pp 8 --micro 32 --mb 16 --only micro --steps 3 --warmup 1 > gpurun_out/prof_ppm.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ppf -o run -- python -u bench/pp_stage_proxy.py --model gpt2-medium --pp 8 --micro 32 --mb 16 --only full --steps 3 --warmup 1 > gpurun_out/prof_ppf.log 2>&1 || exit $?
