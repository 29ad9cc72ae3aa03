#!/bin/bash
# round 6 job 9: attn_fwd3_kernel (the forward's tile loop split by kind, DPC_ATTN_VAR 9 / 10)
# against the shipped attn_fwd2_kernel (6 / 5): numerics (every attention test), forward timing
# interleaved per process, VALU / MFMA instruction counts
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 9 10; do
  DPC_ATTN_VAR=$v,1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 \
    --timeout-method thread -k "attention or attn" > gpurun_out/r6_attn3_t$v.log 2>&1 \
    || { tail -30 gpurun_out/r6_attn3_t$v.log; exit 3; }
  tail -1 gpurun_out/r6_attn3_t$v.log
done
for r in 1 2 3; do
  for v in 6 9 5 10; do
    echo -n "var $v: "; DPC_ATTN_VAR=$v,1 timeout -k 10 120 python -u bench/attn_time.py --rounds 5 --iters 10 2>/dev/null \
      | grep '^{' || exit 4
  done
done | tee gpurun_out/r6_attn3_var.log || exit 4
for v in 6 9; do
  DPC_ATTN_VAR=$v,1 timeout -k 10 100 scripts/pmc_attn_c.sh a3v$v > gpurun_out/r6_pmc_a3v$v.log 2>&1 || exit 5
  echo "== var $v"; python scripts/pmc_summary.py gpurun_out/pmc_a3v${v}_c/p_results.db attn_fwd
done
