#!/bin/bash
# Same-box A/B of the LDS-staged act' epilogue + packed GELU + re-tuned table (new) against the
# previous table with the per-lane act' reads (old: DPC_GEMM_TABLE_PATH=gpurun_old_table.json,
# DPC_G7_ACTLDS=0), alternating processes, on the four recipe benches.  gpurun_old_table.json:
# git show <previous commit>:distributed_pytorch_cookbook_amd/ops/gemm_tuned.json
OLD="DPC_GEMM_TABLE_PATH=gpurun_old_table.json DPC_G7_ACTLDS=0"
scripts/gpu_step.sh \
  "150:ab_ddp_new1:python -u bench.py" "150:ab_ddp_old1:env $OLD python -u bench.py" \
  "150:ab_ddp_new2:python -u bench.py" "150:ab_ddp_old2:env $OLD python -u bench.py" \
  "200:ab_fsdp_new1:python -u bench.py --recipe fsdp --steps 8 --warmup 3" \
  "200:ab_fsdp_old1:env $OLD python -u bench.py --recipe fsdp --steps 8 --warmup 3" \
  "200:ab_fsdp_new2:python -u bench.py --recipe fsdp --steps 8 --warmup 3" \
  "200:ab_fsdp_old2:env $OLD python -u bench.py --recipe fsdp --steps 8 --warmup 3" \
  "200:ab_pipe_new1:python -u bench.py --recipe pipe --steps 8 --warmup 3" \
  "200:ab_pipe_old1:env $OLD python -u bench.py --recipe pipe --steps 8 --warmup 3" \
  "200:ab_ppd_new1:python -u bench.py --recipe pipe_ddp --steps 8 --warmup 3" \
  "200:ab_ppd_old1:env $OLD python -u bench.py --recipe pipe_ddp --steps 8 --warmup 3"
rc=$?
grep -h '"metric"' gpurun_out/ab_*_*[12].log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config']['model'], d['config'].get('parallelism'), d['value'])
" ; exit $rc
