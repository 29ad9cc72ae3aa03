#!/bin/bash
T="python -u -m pytest tests/test_kernels_gpu.py -q --timeout 120 --timeout-method thread -k test_gemm_v6_v7 -p no:randomly"
scripts/gpu_step.sh "200:v67_default:$T" "200:v67_oldepi:env DPC_G7_DEBUG=16 $T" "200:v67_nopair:env DPC_G7_PAIR=0 $T" "200:v67_default2:$T"
