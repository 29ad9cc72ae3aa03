#!/bin/bash
# round 6 job 7: attention forward without the lazy-rescale branch (DPC_ATTN_VAR 9 / 10 against the
# shipped 6 / 5): numerics at hd 64 (fwd + bwd vs f32), then forward timing interleaved per process
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 9 10; do
  DPC_ATTN_VAR=$v,1 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 \
    --timeout-method thread -k "attention_fwd_bwd or attention_long" > gpurun_out/r6_attn_t$v.log 2>&1 \
    || { tail -20 gpurun_out/r6_attn_t$v.log; exit 3; }
  tail -1 gpurun_out/r6_attn_t$v.log
done
for r in 1 2 3; do
  for v in 6 9 5 10; do
    echo -n "var $v: "; DPC_ATTN_VAR=$v,1 timeout -k 10 120 python -u bench/attn_time.py --rounds 5 --iters 10 2>/dev/null \
      | grep '^{' || exit 4
  done
done | tee gpurun_out/r6_attn_var.log
