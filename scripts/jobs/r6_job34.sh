#!/bin/bash
# round 6 job 34: IPC copy-only collectives of any dtype (the pipeline's int64 generation
# broadcast): the IPC tests, then the multi-rank script options of job 33
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/jobs/r6_job12.sh > gpurun_out/r6_ipc34.txt 2>&1 || { tail -30 gpurun_out/r6_ipc34.txt; exit 3; }
grep -E "passed|failed" gpurun_out/r6_ipc34.txt | tail -1
scripts/jobs/r6_job33.sh
