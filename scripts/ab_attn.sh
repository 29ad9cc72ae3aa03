#!/bin/bash
# A/B the attention kernels: the in-tree library vs a saved previous build (bench/*.bak).
scripts/gpu_step.sh "200:attn_t:python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k attention" \
  "60:new_f:python bench/attn_one.py --N 64 --iters 20" "60:new_b:python bench/attn_one.py --N 64 --iters 10 --bwd" \
  "150:new_bench:python -u bench.py --steps 10" || exit $?
cp distributed_pytorch_cookbook_amd/ops/libdpc_kernels.so gpurun_out/new.so
cp bench/libdpc_kernels_old.so.bak distributed_pytorch_cookbook_amd/ops/libdpc_kernels.so
scripts/gpu_step.sh "60:old_f:python bench/attn_one.py --N 64 --iters 20" "60:old_b:python bench/attn_one.py --N 64 --iters 10 --bwd" \
  "150:old_bench:python -u bench.py --steps 10"
