#!/bin/bash
# GPU tests after the round-4 GEMM changes, a full re-timing of the GEMM table with nt stores
# (bench/retune_keys.py, auto timed through the table), then the recipe benches on the old and
# the re-timed table, alternating
scripts/gpu_step.sh "500:gputests:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" || exit $?
scripts/gpu_step.sh "900:retune:python -u bench/retune_keys.py --match . --impls 0 2 3 4 10 12 16 19 20 21 22 23 24 25 26 --write gpurun_out/gemm_tuned_r4.json" || exit $?
T=distributed_pytorch_cookbook_amd/ops/gemm_tuned.json
for i in 1 2; do
  scripts/gpu_step.sh "150:b_ddp_old_$i:python -u bench.py" \
    "150:b_ddp_new_$i:DPC_GEMM_TABLE_PATH=gpurun_out/gemm_tuned_r4.json python -u bench.py" || exit $?
done
for r in fsdp pipe pipe_ddp; do
  scripts/gpu_step.sh "200:b_${r}_old:python -u bench.py --recipe $r --steps 8 --warmup 3" \
    "200:b_${r}_new:DPC_GEMM_TABLE_PATH=gpurun_out/gemm_tuned_r4.json python -u bench.py --recipe $r --steps 8 --warmup 3" || exit $?
done
grep -h '"value"' gpurun_out/b_*_old*.log gpurun_out/b_*_new*.log | python3 -c "
import sys, json
for l in sys.stdin: d = json.loads(l); print(d['config']['recipe'], d['value'], d['ms_per_step'])"
# one-GPU proxies of the pipeline north stars (PP=8 GPT-2 medium, PP=2 GPT-2 large)
scripts/gpu_step.sh "300:pp8_medium_fp32:python -u bench/pp_stage_proxy.py --model gpt2-medium --pp 8 --micro 32 --mb 16 --graph --json gpurun_out/pp8_medium_fp32.json" \
  "300:pp8_medium_bf16:python -u bench/pp_stage_proxy.py --model gpt2-medium --pp 8 --micro 32 --mb 16 --wire bf16 --json gpurun_out/pp8_medium_bf16.json" \
  "300:pp2_large_fp32:python -u bench/pp_stage_proxy.py --model gpt2-large --pp 2 --micro 8 --mb 16 --graph --json gpurun_out/pp2_large_fp32.json"
