#!/bin/bash
# nt epilogue stores: GEMM tests, then the DDP bench alternating DPC_GEMM_NT=3 / 0 / 1, and the
# per-product A/B against hipBLASLt with the default (nt) mode
scripts/gpu_step.sh "300:gemmtests:python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_table_gpu.py -x -q -k 'gemm or g7 or g9 or table' --timeout 120 --timeout-method thread" || exit $?
for i in 1 2; do
  for m in 3 0 1; do
    scripts/gpu_step.sh "150:b_nt${m}_$i:DPC_GEMM_NT=$m python -u bench.py" || exit $?
  done
done
scripts/gpu_step.sh "300:gemm_ab_nt:python -u bench/gemm_ab.py --shapes gpt2s --rounds 3" \
  "300:gemm_ab_fused_nt:python -u bench/gemm_ab.py --shapes fused --rounds 3"
grep -h '"value"' gpurun_out/b_nt*.log | python3 -c "
import sys, json
for l in sys.stdin: d = json.loads(l); print(d['value'], d['ms_per_step'])"
