#!/bin/bash
# final state of the round: full GPU tests, smoke, the four benches, DDP kernel table
scripts/gpu_step.sh "300:warm:python -u scripts/warm.py" \
  "700:gputests:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200:smoke:python -u -c 'import __graft_entry__ as g; g.smoke()'" || exit $?
i=0
for r in ddp ddp fsdp pipe pipe_ddp; do
  i=$((i + 1))
  scripts/gpu_step.sh "200:fb_${i}_${r}:python -u bench.py --recipe $r" || exit $?
done
grep -h '"value"' gpurun_out/fb_*.log | python3 -c '
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d["config"]["recipe"], d["config"]["model"], d["value"], d["ms_per_step"], d["config"]["mfu_per_gpu"])'
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run -- python -u bench.py --steps 10 --warmup 3 > gpurun_out/prof_final.log 2>&1 || exit $?
