#!/bin/bash
# long-context throughput on the round-4 tree (64K tokens per step, S = 2K / 4K / 8K) and the
# FSDP XL kernel table
scripts/gpu_step.sh "300:warm:python -u scripts/warm.py" \
  "150:lc_s2048:python -u bench.py --seq_len 2048 --batch_size 32 --steps 10 --warmup 3" \
  "150:lc_s4096:python -u bench.py --seq_len 4096 --batch_size 16 --steps 10 --warmup 3" \
  "150:lc_s8192:python -u bench.py --seq_len 8192 --batch_size 8 --steps 10 --warmup 3" || exit $?
grep -h '"value"' gpurun_out/lc_s*.log | python3 -c '
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d["config"]["seq_len"], d["value"], d["ms_per_step"], d["config"]["mfu_per_gpu"])'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fsdp -o run -- python -u bench.py --recipe fsdp --steps 4 --warmup 2 > gpurun_out/prof_fsdp.log 2>&1 || exit $?
