#!/bin/bash
# Same-box A/B of two GEMM tables: A = $TA, B = the in-package table; DDP and FSDP benches alternated.
for r in 1 2; do
  DPC_GEMM_TABLE_PATH=$TA timeout -k 10 150 python -u bench.py 2>&1 | grep -o '"value": [0-9.]*' | sed "s/^/A ddp /" || exit 1
  timeout -k 10 150 python -u bench.py 2>&1 | grep -o '"value": [0-9.]*' | sed "s/^/B ddp /" || exit 1
done
for r in 1 2; do
  DPC_GEMM_TABLE_PATH=$TA timeout -k 10 200 python -u bench.py --recipe fsdp --steps 8 --warmup 3 2>&1 | grep -o '"value": [0-9.]*' | sed "s/^/A fsdp /" || exit 1
  timeout -k 10 200 python -u bench.py --recipe fsdp --steps 8 --warmup 3 2>&1 | grep -o '"value": [0-9.]*' | sed "s/^/B fsdp /" || exit 1
done
