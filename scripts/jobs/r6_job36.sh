#!/bin/bash
# round 6 job 36: bench.py FSDP at N = 2 on one GPU over IPC with the step graph (GPT-2 medium, 16
# sequences per rank; a rehearsal of the FSDP N > 1 graphed bench path -- no throughput result)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DPC_DIST_BACKEND=gloo DPC_IPC_SPIN=8000000
timeout -k 10 300 python -u bench.py --gpus 2 --comm ipc --graph --recipe fsdp --model gpt2-medium --batch_size 16 \
  --steps 4 --warmup 3 > gpurun_out/r6_n2_fsdp_medium.log 2>&1
rc=$?
echo "rc=$rc"; grep '^{' gpurun_out/r6_n2_fsdp_medium.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); c=d['config']
    print({k: d[k] for k in ('value','ms_per_step','n_gpus')}, {k: c.get(k) for k in ('model','parallelism','comm','step_graph','final_loss')})"
exit $rc
