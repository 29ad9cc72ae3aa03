#!/bin/bash
# Numerics (attention tests) + timing of forward variants given as VARS (DPC_ATTN_VAR fwd part).
for v in ${VARS:-5 6}; do
  DPC_ATTN_VAR=$v,1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attention 2>&1 | tail -2 | sed "s/^/var$v tests: /" || exit $?
done
for hd in 64 32; do for v in 0 2 ${VARS:-5 6}; do
  DPC_ATTN_VAR=$v,1 timeout -k 5 60 python -u bench/attn_one.py --N 64 --S 1023 --H 12 --hd $hd --iters 20 2>&1 | grep us | sed "s/^/var$v /" || exit $?
done; done
