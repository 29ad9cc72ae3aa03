#!/bin/bash
# round-4 state: GEMM / table tests, pipeline stage proxies after the weight-gradient policy fix,
# LayerNorm backward grid sweep at the micro-batch shapes, every recipe's bench, full GPU tests,
# smoke
scripts/gpu_step.sh "300:warm:python -u scripts/warm.py" \
  "300:t_gemm:python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_table_gpu.py -x -q --timeout 120 --timeout-method thread -k 'gemm or table'" \
  "300:pp8_medium:python -u bench/pp_stage_proxy.py --model gpt2-medium --pp 8 --micro 32 --mb 16 --graph --json gpurun_out/pp8_medium_r4b.json" \
  "300:pp2_large:python -u bench/pp_stage_proxy.py --model gpt2-large --pp 2 --micro 8 --mb 16 --json gpurun_out/pp2_large_r4b.json" \
  "200:ln_grid:python -u bench/ln_grid.py 16368x1024,16368x1280,65472x1024,65472x768" || exit $?
i=0
for r in ddp ddp fsdp pipe pipe_ddp; do
  i=$((i + 1))
  scripts/gpu_step.sh "200:bench_${i}_${r}:python -u bench.py --recipe $r" || exit $?
done
grep -h '"value"' gpurun_out/bench_*.log | python3 -c '
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d["config"]["recipe"], d["config"]["model"], d["value"], d["ms_per_step"], d["config"]["mfu_per_gpu"])'
scripts/gpu_step.sh "700:gputests:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200:smoke:python -u -c 'import __graft_entry__ as g; g.smoke()'" || exit $?
