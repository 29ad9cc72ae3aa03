#!/bin/bash
# v9 split-K slabs for the weight gradients: GEMM GPU tests, then v9 (default) vs v7
# (DPC_G9_WGRAD=0) on the GPT-2 small / XL weight gradients and the bench, alternating processes.
scripts/gpu_step.sh "300:gemmtests:python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_table_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread" || exit $?
for rep in 1 2; do
  scripts/gpu_step.sh "200:w_on_$rep:python -u bench/gemm_ab.py --shapes wgrad --impls 25 --rounds 3" \
    "200:w_off_$rep:DPC_G9_WGRAD=0 python -u bench/gemm_ab.py --shapes wgrad --impls 25 --rounds 3" \
    "200:b_on_$rep:python -u bench.py" "200:b_off_$rep:DPC_G9_WGRAD=0 python -u bench.py" || exit $?
done
scripts/gpu_step.sh "300:x_on:python -u bench/gemm_ab.py --shapes xl --impls 25 --only xl_w_qkv xl_w_out xl_w_up xl_w_down xl_w_lm --rounds 3" \
  "300:x_off:DPC_G9_WGRAD=0 python -u bench/gemm_ab.py --shapes xl --impls 25 --only xl_w_qkv xl_w_out xl_w_up xl_w_down xl_w_lm --rounds 3"
for f in b_on_1 b_off_1 b_on_2 b_off_2; do echo -n "$f: "; grep -o '"value": [0-9.]*' gpurun_out/$f.log; done
