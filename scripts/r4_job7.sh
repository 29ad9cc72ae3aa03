#!/bin/bash
# cross-entropy with one exponential per logit (DPC_CE_MODE=3): numerics, kernel A/B, DDP A/B
scripts/gpu_step.sh "300:warm:python -u scripts/warm.py" \
  "200:t_ce:python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k cross_entropy" \
  "120:ce_one:python -u bench/ce_one.py" || exit $?
for i in 1 2 3; do
  scripts/gpu_step.sh "150:h_ce0_$i:DPC_CE_MODE=0 python -u bench.py" "150:h_ce3_$i:DPC_CE_MODE=3 python -u bench.py" || exit $?
done
for f in gpurun_out/h_*.log; do
  echo "$f $(grep -h '"value"' $f | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])')"
done
