#!/bin/bash
# round 6 job 12: peer-access (HIP IPC) collectives, two ranks sharing the GPU: every collective
# exact, graph replays, DDP / FSDP over the IPC transport with the step captured on both ranks
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_ipc_gpu.py -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/r6_ipc12.log 2>&1
rc=$?
tail -40 gpurun_out/r6_ipc12.log
exit $rc
