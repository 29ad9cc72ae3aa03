#!/bin/bash
# round 6 job 33: multi-rank options on the one GPU over the IPC transport: collective generation
# (FSDP, pipeline), --coll_check, FSDP --cpu_offload
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DPC_IPC_SPIN=4000000 DPC_DIST_BACKEND=gloo
A="--synthetic_data --epochs 1 --max_steps 16 --num_workers 0 --no_save --comm ipc"
port=29770
run() {
  local name=$1 n=$2; shift 2
  port=$((port + 1))
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $port "$@" > gpurun_out/r6_mr_$name.log 2>&1
  local rc=$?
  local last=$(tr '\r' '\n' < gpurun_out/r6_mr_$name.log | grep -E "\[training\]" | grep -v "?????" | tail -1 | sed 's/|[^|]*it\/s\]//' | cut -c1-100)
  echo "$name rc=$rc | $last | $(grep -E '^\[validation\]' gpurun_out/r6_mr_$name.log | tail -1)"
  grep -c "Argmax sampling" gpurun_out/r6_mr_$name.log
  return $rc
}
run fsdp_generate 2 main-fsdp.py $A || exit $?
run pipe_generate 2 main-pipe.py $A || exit $?
run ddp_coll_check 2 main-ddp.py $A --no_generate --coll_check || exit $?
run fsdp_offload 2 main-fsdp.py $A --no_generate --cpu_offload || exit $?
