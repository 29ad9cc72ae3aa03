#!/bin/bash
# round 6 job 26: the LayerNorm-feeding input gradients (QKV / FFN up dgrads) in f32, split along
# K, below half a chip of tiles: reference CLI default model A/B, model / engine GPU tests
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_step.sh "400:t26:python -u -m pytest tests/test_model_gpu.py tests/test_engines_gpu.py tests/test_parallel_gpu.py tests/test_fp32_gpu.py -q --timeout 150 --timeout-method thread" || exit $?
grep -q " passed" gpurun_out/t26.log && ! grep -q "FAILED" gpurun_out/t26.log || exit 3
B="python -u bench.py --model ref --seq_len 256 --batch_size 64 --steps 50 --warmup 10"
for r in 1 2 3; do
  echo -n "ln-bf16: "; DPC_LN_DGRAD_F32=0 timeout -k 10 120 $B 2>/dev/null | grep -o '"value": [0-9.]*' || exit 4
  echo -n "auto:    "; timeout -k 10 120 $B 2>/dev/null | grep -o '"value": [0-9.]*' || exit 4
done | tee gpurun_out/r6_ln_dgrad_ab.log
