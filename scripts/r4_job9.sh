#!/bin/bash
# split-K reduction with four slab loads in flight: split-K / weight-gradient tests, kernel
# table, same-box DDP A/B against HEAD (ab_old/)
R=$PWD
scripts/gpu_step.sh "300:warm:python -u scripts/warm.py" \
  "300:t_split:python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_table_gpu.py -x -q --timeout 120 --timeout-method thread -k 'split or wgrad or v7_v8_v9 or table'" || exit $?
(cd ab_old && timeout -k 10 300 python -u ../scripts/warm.py > $R/gpurun_out/warm_old.log 2>&1) || exit $?
for rep in 1 2 3; do
  (cd ab_old && timeout -k 10 150 python -u bench.py > $R/gpurun_out/k_old_$rep.log 2>&1) || exit $?
  timeout -k 10 150 python -u bench.py > gpurun_out/k_new_$rep.log 2>&1 || exit $?
done
for f in gpurun_out/k_*.log; do
  echo "$f $(grep -h '"value"' $f | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_red -o run -- python -u bench.py --steps 10 --warmup 3 > gpurun_out/prof_red.log 2>&1 || exit $?
