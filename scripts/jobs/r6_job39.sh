#!/bin/bash
# round 6 job 39: stability of the multi-process IPC GPU tests (several ranks sharing the one GPU):
# the file three times in a row, each run under its own limit, stopping at the first failure
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2 3; do
  timeout -k 10 420 python -u -m pytest tests/test_ipc_gpu.py -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r6_ipc_stability_$i.log 2>&1 || { echo "run $i failed rc=$?"; tail -30 gpurun_out/r6_ipc_stability_$i.log; exit 1; }
  echo "run $i: $(tail -1 gpurun_out/r6_ipc_stability_$i.log)"
done
