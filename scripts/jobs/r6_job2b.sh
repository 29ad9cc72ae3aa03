#!/bin/bash
# round 6 job 2b: probe the v9 forward epilogue for unwritten / non-finite outputs, then job 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -u bench/nan_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r6_nan_probe.log || exit 5
exec_job2() { bash scripts/jobs/r6_job2.sh; }
exec_job2
