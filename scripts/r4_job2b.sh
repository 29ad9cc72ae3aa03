#!/bin/bash
# GPU tests, GEMM table re-timing with nt stores (+ the chosen v9 schedule), recipe A/B old vs new
# table, attention PMC counters
[ -n "$ER" ] && export DPC_G9_ER=$ER
scripts/gpu_step.sh "300:warm:python -u scripts/warm.py" "200:attn_tests_b:python -u -m pytest tests/test_kernels_gpu.py -x -q -k attention --timeout 120 --timeout-method thread" || exit $?
for i in 1 2; do
  scripts/gpu_step.sh "60:ab_bwd_00_$i:DPC_ATTN_DQ2=0 DPC_ATTN_DKDV2=0 python -u bench/attn_one.py --N 64 --S 1023 --H 12 --iters 20 --bwd" \
    "60:ab_bwd_10_$i:DPC_ATTN_DQ2=1 DPC_ATTN_DKDV2=0 python -u bench/attn_one.py --N 64 --S 1023 --H 12 --iters 20 --bwd" \
    "60:ab_bwd_11_$i:DPC_ATTN_DQ2=1 DPC_ATTN_DKDV2=1 python -u bench/attn_one.py --N 64 --S 1023 --H 12 --iters 20 --bwd" || exit $?
done
DPC_ATTN_DQ2=1 DPC_ATTN_DKDV2=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dq2 -o run -- python -u bench/attn_one.py --N 64 --S 1023 --H 12 --iters 10 --bwd > gpurun_out/prof_dq2.log 2>&1 || exit $?
[ -n "$DQ2" ] && export DPC_ATTN_DQ2=$DQ2
[ -n "$DKDV2" ] && export DPC_ATTN_DKDV2=$DKDV2
scripts/gpu_step.sh "500:gputests:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" || exit $?
scripts/gpu_step.sh "900:retune:python -u bench/retune_keys.py --match . --impls 0 2 3 4 10 12 16 19 20 21 22 23 24 25 26 --write gpurun_out/gemm_tuned_r4.json" || exit $?
for i in 1 2; do
  scripts/gpu_step.sh "150:t_ddp_old_$i:python -u bench.py" \
    "150:t_ddp_new_$i:DPC_GEMM_TABLE_PATH=gpurun_out/gemm_tuned_r4.json python -u bench.py" || exit $?
done
for r in fsdp pipe pipe_ddp; do
  scripts/gpu_step.sh "200:t_${r}_old:python -u bench.py --recipe $r --steps 8 --warmup 3" \
    "200:t_${r}_new:DPC_GEMM_TABLE_PATH=gpurun_out/gemm_tuned_r4.json python -u bench.py --recipe $r --steps 8 --warmup 3" || exit $?
done
for f in gpurun_out/t_*.log; do
  echo "$f $(grep -h '"value"' $f | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 bash scripts/pmc_attn_all.sh > gpurun_out/pmc_attn.log 2>&1
cat gpurun_out/pmc_attn_summary.txt
