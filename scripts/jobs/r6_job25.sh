#!/bin/bash
# round 6 job 25: the LM-head input gradient in f32 (split along K) when it is under half a chip of
# tiles -- the reference CLI default model (D 256): A/B against the bf16 form, the model / engine
# GPU tests, and GPT-2 small unchanged (its product is 768 tiles)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_step.sh "400:t25:python -u -m pytest tests/test_model_gpu.py tests/test_engines_gpu.py tests/test_parallel_gpu.py -q --timeout 150 --timeout-method thread" || exit $?
grep -q " passed" gpurun_out/t25.log && ! grep -q "FAILED" gpurun_out/t25.log || exit 3
B="python -u bench.py --model ref --seq_len 256 --batch_size 64 --steps 50 --warmup 10"
for r in 1 2 3; do
  echo -n "bf16: "; DPC_HEAD_DGRAD_F32=0 timeout -k 10 120 $B 2>/dev/null | grep -o '"value": [0-9.]*' || exit 4
  echo -n "auto: "; timeout -k 10 120 $B 2>/dev/null | grep -o '"value": [0-9.]*' || exit 4
done | tee gpurun_out/r6_head_dgrad_ab.log
echo -n "gpt2-small auto: "; timeout -k 10 200 python -u bench.py 2>/dev/null | grep -o '"value": [0-9.]*'
