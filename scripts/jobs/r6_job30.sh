#!/bin/bash
# round 6 job 30: main-pipe.py (2 stages, 1F1B) at N = 2 on the one GPU over the IPC transport -- a
# probe of the shared-GPU co-residency stall seen with GPT-2 medium (profiles/r6_ipc/README.md)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
A="--synthetic_data --epochs 1 --max_steps 20 --no_save --num_workers 0 --no_generate"
DPC_IPC_SPIN=4000000 DPC_DIST_BACKEND=gloo timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29741 main-pipe.py $A --comm ipc > gpurun_out/r6_cli_main-pipe_2.log 2>&1
rc=$?
echo "rc=$rc"; grep -v "socket.cpp\|Gloo\]\|amdgpu.ids\|W1019" gpurun_out/r6_cli_main-pipe_2.log | tr '\r' '\n' | grep -v "?????" | tail -6
