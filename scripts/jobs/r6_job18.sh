#!/bin/bash
# round 6 job 18: the IPC point-to-point half-reuse fix (a sender now waits for the ACKs of every
# workgroup of the receiver): the IPC tests three times over (the race was intermittent), then the
# whole GPU suite
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for k in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_ipc_gpu.py -x -q --timeout 150 --timeout-method thread \
    > gpurun_out/r6_ipc18_$k.log 2>&1 || { tail -30 gpurun_out/r6_ipc18_$k.log; exit 3; }
  tail -1 gpurun_out/r6_ipc18_$k.log
done
scripts/gpu_step.sh "600:r6_gputests18:python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread" || exit $?
grep -q " passed" gpurun_out/r6_gputests18.log && ! grep -q "FAILED" gpurun_out/r6_gputests18.log
