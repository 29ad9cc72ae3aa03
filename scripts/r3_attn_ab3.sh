#!/bin/bash
# dK/dV kernel with its K / V rows by LDS-DMA (ring slots 2 / 3) instead of per-lane 16-B row loads:
# attention numerics tests, then old (ab_old/, HEAD) vs new backward timing, alternating processes.
scripts/gpu_step.sh "300:t_attn:python -u -m pytest tests/test_kernels_gpu.py tests/test_fp32_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -k 'attention or attn or model'" || exit $?
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export DPC_ROOT=ab_old; else unset DPC_ROOT; fi
    for cfg in "--hd 64 --H 12" "--hd 32 --H 24" "--hd 64 --H 25"; do
      echo -n "$v $cfg --bwd: "
      timeout -k 10 60 python -u bench/attn_one.py --N 64 --S 1023 --iters 20 $cfg --bwd 2>/dev/null | tail -1 || exit $?
    done
  done
done
