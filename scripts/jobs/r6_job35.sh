#!/bin/bash
# round 6 job 35: multi-rank save / resume over IPC (FSDP N = 2, pipeline N = 2), --stream_check at
# N = 2, main-pipe-ddp.py N = 4 with generation
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DPC_IPC_SPIN=4000000 DPC_DIST_BACKEND=gloo
A="--synthetic_data --epochs 1 --num_workers 0 --comm ipc"
port=29790
run() {
  local name=$1 n=$2; shift 2
  port=$((port + 1))
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $port "$@" > gpurun_out/r6_mr_$name.log 2>&1
  local rc=$?
  local last=$(tr '\r' '\n' < gpurun_out/r6_mr_$name.log | grep -E "\[training\]" | grep -v "?????" | tail -1 | sed 's/|[^|]*it\/s\]//' | cut -c1-100)
  echo "$name rc=$rc | $last | $(grep -E '^\[validation\]' gpurun_out/r6_mr_$name.log | tail -1) | $(grep -E '^\[resume\]' gpurun_out/r6_mr_$name.log | head -1)"
  return $rc
}
for s in main-fsdp.py main-pipe.py; do
  b=${s%.py}
  run ${b}_save 2 $s $A --max_steps 12 --no_generate --checkpoint_dir gpurun_out/ck35_$b --save_every 6 || exit $?
  ls gpurun_out/ck35_$b | head -5
  # a second epoch from the saved state: --epochs 2 resumes after epoch 1
  run ${b}_resume 2 $s --synthetic_data --epochs 2 --num_workers 0 --comm ipc --max_steps 12 --no_generate \
    --checkpoint_dir gpurun_out/ck35_$b --resume latest || exit $?
  rm -rf gpurun_out/ck35_$b
done
run ddp_stream_check 2 main-ddp.py $A --max_steps 12 --no_save --no_generate --stream_check || exit $?
run ppd_generate 4 main-pipe-ddp.py $A --max_steps 12 --no_save || exit $?
grep -c "Argmax sampling" gpurun_out/r6_mr_ppd_generate.log
