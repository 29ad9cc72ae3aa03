#!/bin/bash
# v9 for the plain input gradients (impl 26 A/B against the table), v9's forward epilogue with
# the early-release schedule (DPC_G9_FWD_ER=4)
scripts/gpu_step.sh "300:warm:python -u scripts/warm.py" \
  "300:t_v9:python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k 'v7_v8_v9 or v9_forward'" \
  "300:t_v9_er:DPC_G9_FWD_ER=4 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k 'v9_forward'" \
  "200:ab_gpt2s:python -u bench/gemm_ab.py --shapes gpt2s --impls 20 26" \
  "200:ab_xl:python -u bench/gemm_ab.py --shapes xl --impls 20 26" \
  "200:ab_fused_er0:python -u bench/gemm_ab.py --shapes fused --impls 26" \
  "200:ab_fused_er4:DPC_G9_FWD_ER=4 python -u bench/gemm_ab.py --shapes fused --impls 26" || exit $?
for i in 1 2 3; do
  scripts/gpu_step.sh "150:g_base_$i:python -u bench.py" "150:g_fer4_$i:DPC_G9_FWD_ER=4 python -u bench.py" || exit $?
done
scripts/gpu_step.sh "200:g_fsdp_base:python -u bench.py --recipe fsdp --steps 6 --warmup 2" \
  "200:g_fsdp_fer4:DPC_G9_FWD_ER=4 python -u bench.py --recipe fsdp --steps 6 --warmup 2" || exit $?
for f in gpurun_out/g_*.log; do
  echo "$f $(grep -h '"value"' $f | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
