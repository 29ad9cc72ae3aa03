#!/bin/bash
# v9 forward epilogue + scalar alpha + ER 4 default: tests, fused-GEMM A/B, DDP A/B with the
# up-projection on v9; dQ pair stream A/B; table re-timing; full GPU tests; attention PMC
scripts/gpu_step.sh "300:warm:python -u scripts/warm.py" \
  "300:t_new:python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'attention or v9_forward or v7_v8_v9' --timeout 120 --timeout-method thread" || exit $?
scripts/gpu_step.sh "200:ab_fused:python -u bench/gemm_ab.py --shapes fused --impls 10 24 26" || exit $?
for i in 1 2; do
  scripts/gpu_step.sh "150:d_base_$i:python -u bench.py" \
    "150:d_g9fwd_$i:DPC_GEMM_TABLE_PATH=bench/tables/gemm_tuned_g9fwd.json python -u bench.py" \
    "150:d_dq2_$i:DPC_ATTN_DQ2=1 python -u bench.py" || exit $?
done
for f in gpurun_out/d_*.log; do
  echo "$f $(grep -h '"value"' $f | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
for i in 1 2; do
  scripts/gpu_step.sh "60:ab_bwd_00_$i:DPC_ATTN_DQ2=0 DPC_ATTN_DKDV2=0 python -u bench/attn_one.py --N 64 --S 1023 --H 12 --iters 20 --bwd" \
    "60:ab_bwd_10_$i:DPC_ATTN_DQ2=1 DPC_ATTN_DKDV2=0 python -u bench/attn_one.py --N 64 --S 1023 --H 12 --iters 20 --bwd" || exit $?
done
DPC_ATTN_DQ2=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dq2 -o run -- python -u bench/attn_one.py --N 64 --S 1023 --H 12 --iters 10 --bwd > gpurun_out/prof_dq2.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ddp -o run -- python -u bench.py --steps 10 --warmup 3 > gpurun_out/prof_ddp.log 2>&1 || exit $?
scripts/gpu_step.sh "300:pp2_large_fp32:python -u bench/pp_stage_proxy.py --model gpt2-large --pp 2 --micro 8 --mb 16 --graph --json gpurun_out/pp2_large_fp32.json" || exit $?
scripts/gpu_step.sh "600:gputests:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" || exit $?
