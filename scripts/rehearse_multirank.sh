#!/bin/bash
# Rehearse the multi-rank GPU paths of bench.py on a ONE-GPU box: several ranks share
# cuda:0 and talk over gloo (DPC_DIST_BACKEND=gloo; RCCL refuses two ranks per GPU), so
# the engines' bucketing / sharding / pipeline scheduling run with the real HIP kernels.
# Throughput numbers from this are meaningless (host-staged collectives, shared GPU).
#   scripts/rehearse_multirank.sh [steps]
steps=${1:-3}
export DPC_DIST_BACKEND=gloo
port=29611
run() {  # name nproc args...
  local name=$1 np=$2; shift 2
  port=$((port + 1))
  echo "--- $name (nproc $np)"
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$np" \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus "$np" --steps "$steps" --warmup 1 "$@" \
    > "gpurun_out/rehearse_$name.log" 2>&1
  local rc=$?
  tail -n 3 "gpurun_out/rehearse_$name.log"
  return $rc
}
mkdir -p gpurun_out
run ddp2 2 --batch_size 8 &&
run ddp2_bf16 2 --batch_size 8 --reduce_dtype bf16 &&
run fsdp2 2 --recipe fsdp --model gpt2-medium --batch_size 4 &&
run pipe2 2 --recipe pipe --batch_size 8 &&
run pipe4_gpipe 4 --recipe pipe --batch_size 8 --schedule gpipe &&
run pipeddp4 4 --recipe pipe_ddp --model gpt2-medium --batch_size 4 --dp_size 2 &&
run pipe4_default 4 --recipe pipe --model gpt2-small &&
run pipeddp4_default 4 --recipe pipe_ddp --model gpt2-small
