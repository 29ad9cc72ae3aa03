#!/bin/bash
# the engines' N > 1 code paths at one rank over the native RCCL communicator with bf16 gradient
# reduction (DDP bucket all-reduce, FSDP reduce-scatter, PP x DP stage all-reduce) against fp32
scripts/gpu_step.sh "300:warm:python -u scripts/warm.py" \
  "150:rd_ddp_fp32:python -u bench.py --force_dist_path --reduce_dtype fp32" \
  "150:rd_ddp_bf16:python -u bench.py --force_dist_path --reduce_dtype bf16" \
  "250:rd_fsdp_fp32:python -u bench.py --recipe fsdp --force_dist_path --reduce_dtype fp32 --steps 6 --warmup 2" \
  "250:rd_fsdp_bf16:python -u bench.py --recipe fsdp --force_dist_path --reduce_dtype bf16 --steps 6 --warmup 2" \
  "250:rd_ppdp_fp32:python -u bench.py --recipe pipe_ddp --force_dist_path --reduce_dtype fp32 --steps 8 --warmup 3" \
  "250:rd_ppdp_bf16:python -u bench.py --recipe pipe_ddp --force_dist_path --reduce_dtype bf16 --steps 8 --warmup 3" || exit $?
grep -h '"value"' gpurun_out/rd_*.log | python3 -c '
import sys, json
for l in sys.stdin:
    d = json.loads(l); c = d["config"]
    print(c["recipe"], c.get("reduce_dtype", "?"), d["value"], d["ms_per_step"], c["final_loss"], c["force_dist_path"])'
