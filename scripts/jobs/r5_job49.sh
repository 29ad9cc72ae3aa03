#!/bin/bash
# round 5 job 49: re-time every GPT-2-small step GEMM entry of the table against all candidate
# implementations on today's kernels (store scope 15), then the DDP bench with the old / new table
mkdir -p gpurun_out
timeout -k 10 600 python -u bench/retune_keys.py \
  --match '^(65472x(768|2304|3072|50304)x(768|2304|3072|50304):|(768|2304|3072|50257)x(768|3072)x65472:)' \
  --impls 0 2 3 4 10 16 17 19 20 21 22 23 24 25 26 --write gpurun_out/gemm_tuned_r5.json > gpurun_out/r5_retune.log 2>&1 \
  || { tail -20 gpurun_out/r5_retune.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5_retune.log | cut -c1-220
for r in 1 2; do
  echo "== table old"; timeout -k 10 200 python -u bench.py 2>&1 | grep -v amdgpu.ids | sed 's/"unit".*//' || exit 1
  echo "== table new"; DPC_GEMM_TABLE_PATH=gpurun_out/gemm_tuned_r5.json timeout -k 10 200 python -u bench.py 2>&1 | grep -v amdgpu.ids | sed 's/"unit".*//' || exit 1
done
