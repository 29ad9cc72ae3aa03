#!/bin/bash
# v9 early-release lab + DDP A/B, CU co-residency, pipeline proxies
scripts/gpu_step.sh "300:warm:python -u scripts/warm.py" \
  "60:attn_fwd:python -u bench/attn_one.py --N 64 --S 1023 --H 12 --iters 20" \
  "60:attn_bwd:python -u bench/attn_one.py --N 64 --S 1023 --H 12 --iters 20 --bwd" \
  "60:attn_bwd_dkdv2:DPC_ATTN_DKDV2=1 python -u bench/attn_one.py --N 64 --S 1023 --H 12 --iters 20 --bwd" \
  "60:attn_bwd_b:python -u bench/attn_one.py --N 64 --S 1023 --H 12 --iters 20 --bwd" \
  "60:attn_bwd_dkdv2_b:DPC_ATTN_DKDV2=1 python -u bench/attn_one.py --N 64 --S 1023 --H 12 --iters 20 --bwd" \
  "200:attn_tests:python -u -m pytest tests/test_kernels_gpu.py -x -q -k attention --timeout 120 --timeout-method thread" || exit $?
scripts/gpu_step.sh "120:lab_er_qkv:bench/g7lab 65536 2304 768 nt 5 10 er" \
  "120:lab_er_up:bench/g7lab 65536 3072 768 nt 5 10 er" \
  "120:lab_er_lm:bench/g7lab 65536 49152 768 nt 3 3 er" \
  "120:lab_er_sq:bench/g7lab 8192 8192 8192 nt 3 5 er" || exit $?
for i in 1 2; do
  for e in 0 2 4; do
    scripts/gpu_step.sh "150:b_er${e}_$i:DPC_G9_ER=$e python -u bench.py" || exit $?
  done
done
for i in 1 2; do
  scripts/gpu_step.sh "150:b_dkdv2_0_$i:DPC_ATTN_DKDV2=0 python -u bench.py" "150:b_dkdv2_1_$i:DPC_ATTN_DKDV2=1 python -u bench.py" || exit $?
done
for f in gpurun_out/b_er*.log gpurun_out/b_dkdv2*.log; do
  echo "$f $(grep -h '"value"' $f | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
bash scripts/r4_corun.sh || exit $?
scripts/gpu_step.sh "300:pp8_medium_fp32:python -u bench/pp_stage_proxy.py --model gpt2-medium --pp 8 --micro 32 --mb 16 --graph --json gpurun_out/pp8_medium_fp32.json" \
  "300:pp8_medium_bf16:python -u bench/pp_stage_proxy.py --model gpt2-medium --pp 8 --micro 32 --mb 16 --wire bf16 --json gpurun_out/pp8_medium_bf16.json" \
  "300:pp2_large_fp32:python -u bench/pp_stage_proxy.py --model gpt2-large --pp 2 --micro 8 --mb 16 --graph --json gpurun_out/pp2_large_fp32.json"
