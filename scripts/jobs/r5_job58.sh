#!/bin/bash
# round 5 job 58: LayerNorm backward grid size x prefetch
mkdir -p gpurun_out
timeout -k 10 200 python -u bench/ln_bwd_grid2.py 2>&1 | grep -v amdgpu.ids
