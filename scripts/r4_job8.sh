#!/bin/bash
# tune the GEMM signatures the pipeline micro-batches (16 x 1023 tokens) add to the table (the
# weight gradients with K = 16,368 are off-table), then the PP=8 stage proxy with the old and the
# tuned table
scripts/gpu_step.sh "300:warm:python -u scripts/warm.py" \
  "900:tune_pp:DPC_GEMM_TUNE=1 DPC_GEMM_TUNE_OUT=gpurun_out/gemm_tuned_pp.json python -u bench/pp_stage_proxy.py --model gpt2-medium --pp 8 --micro 32 --mb 16 --only micro --steps 1 --warmup 1" || exit $?
python3 - <<'PY'
import json
a = json.load(open("distributed_pytorch_cookbook_amd/ops/gemm_tuned.json"))["impl"]
b = json.load(open("gpurun_out/gemm_tuned_pp.json"))["impl"]
for k in sorted(set(b) - set(a)):
    print("new", k, b[k])
for k in sorted(set(a) & set(b)):
    if a[k] != b[k]:
        print("changed", k, a[k], "->", b[k])
PY
for i in 1 2; do
  scripts/gpu_step.sh "200:pp_old_$i:python -u bench/pp_stage_proxy.py --model gpt2-medium --pp 8 --micro 32 --mb 16 --json gpurun_out/pp_old_$i.json" \
    "200:pp_new_$i:DPC_GEMM_TABLE_PATH=gpurun_out/gemm_tuned_pp.json python -u bench/pp_stage_proxy.py --model gpt2-medium --pp 8 --micro 32 --mb 16 --json gpurun_out/pp_new_$i.json" || exit $?
done
grep -h micro_eager_vs_full gpurun_out/pp_*.json
