#!/bin/bash
# bench.py under several GEMM class policies on the same box (DPC_GEMM_POLICY, csrc/gemm.hip)
#   scripts/policy_sweep.sh "fs=10" "fs=11" ...
for pol in "$@"; do
  echo -n "$pol  "
  DPC_GEMM_POLICY="$pol" timeout -k 10 120 python bench.py --steps 15 --warmup 4 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit $?
done
