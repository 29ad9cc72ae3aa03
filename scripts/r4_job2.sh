#!/bin/bash
# v9 early-release lab + DDP A/B, GPU tests, GEMM table re-timing, recipe A/B, pipeline proxies
scripts/gpu_step.sh "120:lab_er_qkv:bench/g7lab 65536 2304 768 nt 5 10 er" \
  "120:lab_er_up:bench/g7lab 65536 3072 768 nt 5 10 er" \
  "120:lab_er_lm:bench/g7lab 65536 49152 768 nt 3 3 er" \
  "120:lab_er_sq:bench/g7lab 8192 8192 8192 nt 3 5 er" || exit $?
for i in 1 2; do
  for e in 0 2 4; do
    scripts/gpu_step.sh "150:b_er${e}_$i:DPC_G9_ER=$e python -u bench.py" || exit $?
  done
done
best=$(python3 - <<'PY'
import json, glob, collections
v = collections.defaultdict(list)
for f in glob.glob("gpurun_out/b_er*_*.log"):
    e = f.split("b_er")[1].split("_")[0]
    for l in open(f):
        if l.startswith("{"):
            v[e].append(json.loads(l)["value"])
m = {e: sum(x) / len(x) for e, x in v.items()}
print(max(m, key=m.get) if m else 0)
PY
)
echo "best ER = $best"
export DPC_G9_ER=$best
scripts/gpu_step.sh "500:gputests:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" || exit $?
scripts/gpu_step.sh "900:retune:python -u bench/retune_keys.py --match . --impls 0 2 3 4 10 12 16 19 20 21 22 23 24 25 26 --write gpurun_out/gemm_tuned_r4.json" || exit $?
for i in 1 2; do
  scripts/gpu_step.sh "150:b_ddp_old_$i:python -u bench.py" \
    "150:b_ddp_new_$i:DPC_GEMM_TABLE_PATH=gpurun_out/gemm_tuned_r4.json python -u bench.py" || exit $?
done
for r in fsdp pipe pipe_ddp; do
  scripts/gpu_step.sh "200:b_${r}_old:python -u bench.py --recipe $r --steps 8 --warmup 3" \
    "200:b_${r}_new:DPC_GEMM_TABLE_PATH=gpurun_out/gemm_tuned_r4.json python -u bench.py --recipe $r --steps 8 --warmup 3" || exit $?
done
grep -h '"value"' gpurun_out/b_*.log | python3 -c "
import sys, json
for l in sys.stdin: d = json.loads(l); print(d['config']['recipe'], d['value'], d['ms_per_step'])"
bash scripts/r4_corun.sh
scripts/gpu_step.sh "300:pp8_medium_fp32:python -u bench/pp_stage_proxy.py --model gpt2-medium --pp 8 --micro 32 --mb 16 --graph --json gpurun_out/pp8_medium_fp32.json" \
  "300:pp8_medium_bf16:python -u bench/pp_stage_proxy.py --model gpt2-medium --pp 8 --micro 32 --mb 16 --wire bf16 --json gpurun_out/pp8_medium_bf16.json" \
  "300:pp2_large_fp32:python -u bench/pp_stage_proxy.py --model gpt2-large --pp 2 --micro 8 --mb 16 --graph --json gpurun_out/pp2_large_fp32.json"
