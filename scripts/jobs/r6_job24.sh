#!/bin/bash
# round 6 job 24: the reference's own CLI default model (D 256, 8 heads of 32, 8 layers, S 256,
# 64 sequences): its step before / after measuring its GEMM shapes into the table, and its kernels
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="python -u bench.py --model ref --seq_len 256 --batch_size 64 --steps 50 --warmup 10"
scripts/gpu_step.sh "120:ref24_before:$B" || exit $?
export DPC_GEMM_TUNE_OUT=gpurun_out/gemm_tuned.json
cp distributed_pytorch_cookbook_amd/ops/gemm_tuned.json gpurun_out/gemm_tuned.json
DPC_GEMM_TUNE=1 scripts/gpu_step.sh "300:ref24_tune:python -u bench.py --model ref --seq_len 256 --batch_size 64 --steps 2 --warmup 2 --no_graph" || exit $?
python3 - <<'PY'
import json
a = json.load(open("distributed_pytorch_cookbook_amd/ops/gemm_tuned.json"))["impl"]
b = json.load(open("gpurun_out/gemm_tuned.json"))["impl"]
new = {k: v for k, v in b.items() if k not in a}
print("new signatures:", len(new))
for k, v in sorted(new.items()):
    print(f"  {k} -> {v}")
PY
cp gpurun_out/gemm_tuned.json distributed_pytorch_cookbook_amd/ops/gemm_tuned.json
scripts/gpu_step.sh "120:ref24_after:$B" "120:ref24_after2:$B" || exit $?
scripts/prof_bench.sh r6ref --model ref --seq_len 256 --batch_size 64 || exit $?
