#!/bin/bash
# round 6 job 31: main-pipe.py at N = 2 and main-pipe-ddp.py at N = 4 (2 stages x 2 replicas) on the
# one GPU over the IPC transport, after the pipeline loss-logging fix (rank 0 printed nan)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
A="--synthetic_data --epochs 1 --max_steps 24 --no_save --num_workers 0 --no_generate"
for spec in "main-pipe.py:2" "main-pipe-ddp.py:4"; do
  s=${spec%%:*}; n=${spec##*:}
  DPC_IPC_SPIN=4000000 DPC_DIST_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2975$n $s $A --comm ipc > gpurun_out/r6_cli_${s%.py}_$n.log 2>&1 \
    || { tail -30 gpurun_out/r6_cli_${s%.py}_$n.log; exit 4; }
  echo "== $s N=$n ipc"; grep -v "socket.cpp\|Gloo\]\|amdgpu.ids\|W1019" gpurun_out/r6_cli_${s%.py}_$n.log | tr '\r' '\n' | grep -v "?????" | grep -E "training|validation" | tail -3
done
