#!/bin/bash
# round 5 job 63: is the faster 200-step mean a warm state?  20 timed steps after 5 / 50 / 150 warmup
mkdir -p gpurun_out
for w in 5 50 150; do
  echo "== warmup $w"; timeout -k 10 300 python -u bench.py --steps 20 --warmup $w 2>&1 | grep -v amdgpu.ids | grep -o '"value": [0-9.]*\|"final_loss": [0-9.]*' | tr '\n' ' '; echo
done
