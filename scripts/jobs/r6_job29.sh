#!/bin/bash
# round 6 job 29: the user-facing scripts end to end on the GPU -- main-ddp.py at N = 1 (the
# reference's CLI defaults, step graph), then main-ddp.py / main-fsdp.py at N = 2 on the one GPU over
# the peer-access transport (gloo bootstrap), where the recipes now capture the step on every rank
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
A="--synthetic_data --epochs 1 --max_steps 40 --no_save --num_workers 0 --no_generate"
timeout -k 10 240 python -u main-ddp.py $A > gpurun_out/r6_cli_ddp1.log 2>&1 || { tail -20 gpurun_out/r6_cli_ddp1.log; exit 3; }
tail -3 gpurun_out/r6_cli_ddp1.log
for s in main-ddp.py main-fsdp.py; do
  DPC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29731 $s $A --comm ipc > gpurun_out/r6_cli_${s%.py}_2.log 2>&1 \
    || { tail -30 gpurun_out/r6_cli_${s%.py}_2.log; exit 4; }
  echo "== $s N=2 ipc"; grep -v "socket.cpp\|Gloo\]\|amdgpu.ids\|W1019" gpurun_out/r6_cli_${s%.py}_2.log | tail -4
done
