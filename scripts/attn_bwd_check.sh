#!/bin/bash
# Numerics (attention tests) + timing of backward variants given as VARS (DPC_ATTN_VAR bwd part).
for v in ${VARS:-5 6}; do
  DPC_ATTN_VAR=0,$v timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attention 2>&1 | tail -2 | sed "s/^/var$v tests: /" || exit $?
done
for hd in ${HDS:-64 32}; do for v in 1 2 ${VARS:-5 6} 1; do
  DPC_ATTN_VAR=0,$v timeout -k 5 60 python -u bench/attn_one.py --N 64 --S 1023 --H 12 --hd $hd --iters 20 --bwd 2>&1 | grep us | sed "s/^/var$v /" || exit $?
done; done
