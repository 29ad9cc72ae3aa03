#!/bin/bash
# round 6 job 2: GELU' stored by the up-projection forward (aux_deriv) + ACT_MUL input gradient:
# GEMM numerics, model GPU tests, DDP bench against the round-start tree (ab_old) interleaved,
# then the step's kernel trace
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "aux_deriv or act_grad_epilogue or v9_forward or v7_v8_v9 or impls_with_epilogue or v7d or cross_entropy" \
  > gpurun_out/r6j2_tests.log 2>&1 || { tail -30 gpurun_out/r6j2_tests.log; exit 3; }
tail -2 gpurun_out/r6j2_tests.log
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r6j2_model.log 2>&1 || { tail -30 gpurun_out/r6j2_model.log; exit 3; }
tail -2 gpurun_out/r6j2_model.log
for r in 1 2; do
  echo "== new"; timeout -k 10 200 python -u bench.py || exit $?
  echo "== old"; (cd ab_old && timeout -k 10 200 python -u bench.py) || exit $?
done > gpurun_out/r6_bench2.log 2>&1
grep -v amdgpu.ids gpurun_out/r6_bench2.log | sed 's/"unit".*//'
scripts/prof_bench.sh r6s2 || exit $?
# zero-bubble pipeline: the stage proxy with measured F / B / W costs (PP=8 medium, PP=2 large)
for args in "--model gpt2-medium --pp 8 --micro 32 --mb 16" "--model gpt2-medium --pp 8 --micro 16 --mb 32" \
            "--model gpt2-large --pp 2 --micro 8 --mb 16" "--model gpt2-large --pp 2 --micro 4 --mb 32"; do
  for sch in 1f1b zb; do
    timeout -k 10 300 python -u bench/pp_stage_proxy.py $args --schedule $sch --steps 3 --warmup 1 \
      >> gpurun_out/r6_proxy.jsonl 2> gpurun_out/r6_proxy_err.log || { tail -5 gpurun_out/r6_proxy_err.log; exit 4; }
  done
done
cat gpurun_out/r6_proxy.jsonl | python3 -c "import sys,json; [print({k:d.get(k) for k in ('model','pp','micro','mb','micro_eager_vs_full','op_ms','bubble_1f1b','bubble_zb','eff_1f1b','eff_zb')}) for d in map(json.loads, sys.stdin)]"
# PP x DP on the N > 1 code path (one rank): bucket-wise AdamW
timeout -k 10 300 python -u bench.py --recipe pipe_ddp --steps 6 --warmup 2 --force_dist_path > gpurun_out/r6_ppd_fd.log 2>&1 && grep '^{' gpurun_out/r6_ppd_fd.log | cut -c1-150
(cd ab_old && timeout -k 10 300 python -u bench.py --recipe pipe_ddp --steps 6 --warmup 2 --force_dist_path) > gpurun_out/r6_ppd_fd_old.log 2>&1 && grep '^{' gpurun_out/r6_ppd_fd_old.log | cut -c1-150
