#!/bin/bash
# round 6 job 13: peer-access all-reduce latency / local rate (two ranks, one GPU), and the DDP
# bench at N = 2 on one GPU over the IPC transport with the step graph captured on both ranks
# (a rehearsal of the N > 1 graph path: the throughput of two ranks sharing one GPU is no result)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 180 python -u bench/ipc_bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r6_ipc_bench.log || exit $?
DPC_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --comm ipc --graph --steps 6 --warmup 3 \
  > gpurun_out/r6_ipc_bench_n2.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r6_ipc_bench_n2.log | tail -15
exit $rc
