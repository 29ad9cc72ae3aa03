#!/bin/bash
# A/B: measured GEMM table (ops/gemm_tuned.json) vs the dispatcher policy, same box.
scripts/gpu_step.sh "200:ab_ddp0:DPC_GEMM_TABLE=0 python -u bench.py" "200:ab_ddp1:python -u bench.py" \
 "200:ab_fsdp0:DPC_GEMM_TABLE=0 python -u bench.py --recipe fsdp --batch_size 16 --steps 6 --warmup 2" \
 "200:ab_fsdp1:python -u bench.py --recipe fsdp --batch_size 16 --steps 6 --warmup 2" \
 "200:ab_ppd0:DPC_GEMM_TABLE=0 python -u bench.py --recipe pipe_ddp --batch_size 16 --steps 6 --warmup 2" \
 "200:ab_ppd1:python -u bench.py --recipe pipe_ddp --batch_size 16 --steps 6 --warmup 2"
