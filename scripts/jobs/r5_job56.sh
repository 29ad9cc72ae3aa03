#!/bin/bash
# round 5 job 56: the whole GPU suite with the heaviest-first backward order as the default, smoke, bench
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/r5_t56.log 2>&1 \
  || { tail -30 gpurun_out/r5_t56.log; exit 1; }
tail -1 gpurun_out/r5_t56.log
timeout -k 10 120 python -u __graft_entry__.py > gpurun_out/r5_smoke56.log 2>&1 || { tail -20 gpurun_out/r5_smoke56.log; exit 1; }
echo smoke ok
timeout -k 10 200 python -u bench.py 2>&1 | grep -v amdgpu.ids | sed 's/"unit".*//'
