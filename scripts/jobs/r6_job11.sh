#!/bin/bash
# round 6 job 11: GEMM table for the products round 6 changed (the FFN down projection is now a
# bias-only product writing z2: new ':kk:h:00:b' signatures at every model size), measured on the
# four bench recipes; then the recipes again, and a kernel table of FSDP XL
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export DPC_GEMM_TUNE_OUT=gpurun_out/gemm_tuned.json
cp distributed_pytorch_cookbook_amd/ops/gemm_tuned.json gpurun_out/gemm_tuned.json
DPC_GEMM_TUNE=1 scripts/gpu_step.sh "240:t11_ddp:python -u bench.py --steps 2 --warmup 2 --no_graph" \
  "300:t11_fsdp:python -u bench.py --recipe fsdp --steps 2 --warmup 2 --no_graph" \
  "300:t11_pipe:python -u bench.py --recipe pipe --steps 2 --warmup 2 --no_graph" \
  "300:t11_ppd:python -u bench.py --recipe pipe_ddp --steps 2 --warmup 2 --no_graph" || exit $?
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
scripts/gpu_step.sh "150:b11_ddp:python -u bench.py" \
  "200:b11_fsdp:python -u bench.py --recipe fsdp --steps 8 --warmup 3" \
  "200:b11_pipe:python -u bench.py --recipe pipe --steps 8 --warmup 3" \
  "200:b11_ppd:python -u bench.py --recipe pipe_ddp --steps 8 --warmup 3" || exit $?
scripts/prof_bench.sh r6xl --recipe fsdp || exit $?
