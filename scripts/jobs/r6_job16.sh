#!/bin/bash
# round 6 job 16: bench.py at N = 2 on ONE GPU over the peer-access transport with the step graph
# captured on both ranks, every recipe (a rehearsal of the N > 1 graphed paths at real model sizes;
# two ranks share the GPU, so the throughputs are no result).  FSDP at a smaller per-GPU batch: two
# GPT-2 XL ranks at 64 sequences would not fit one GPU's memory together.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DPC_DIST_BACKEND=gloo
run() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --gpus 2 --comm ipc --graph --steps 4 --warmup 3 "$@" \
    > gpurun_out/r6_n2_$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep '^{' gpurun_out/r6_n2_$name.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); c=d['config']
    print({k: d[k] for k in ('value','ms_per_step','n_gpus')}, {k: c.get(k) for k in ('model','parallelism','comm','step_graph','schedule','final_loss')})"
  return $rc
}
run pipe --recipe pipe || exit $?
run ppd --recipe pipe_ddp || exit $?
run fsdp --recipe fsdp --batch_size 16 || exit $?
