#!/bin/bash
# A/B kernel-library builds on one box: for each bench/ab_*.so.bak (and the in-tree build,
# "cur"), run the attention microbenches and a short bench.py.  The in-tree .so is restored.
run_set() {
  scripts/gpu_step.sh "200:${1}_t:python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k attention" \
    "60:${1}_f:python bench/attn_one.py --N 64 --iters 20" \
    "60:${1}_b:python bench/attn_one.py --N 64 --iters 10 --bwd" \
    "150:${1}_bench:python -u bench.py --steps 10"
}
L=distributed_pytorch_cookbook_amd/ops/libdpc_kernels.so
cp $L gpurun_out/cur.so.keep
run_set cur || exit $?
for f in bench/ab_*.so.bak; do
  name=$(basename $f .so.bak)
  cp $f $L
  run_set $name || { cp gpurun_out/cur.so.keep $L; exit 1; }
done
cp gpurun_out/cur.so.keep $L
rm -f gpurun_out/cur.so.keep
