#!/bin/bash
# round 5 job 67: attention GPU tests incl. the block-order bitwise test
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "attn or attention" > gpurun_out/r5_t67.log 2>&1 || { tail -30 gpurun_out/r5_t67.log; exit 1; }
tail -1 gpurun_out/r5_t67.log
