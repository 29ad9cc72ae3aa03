#!/bin/bash
# Multi-GPU tuning sweep for a whole 8 x MI355X node (not runnable on the one-GPU boxes of this
# project's CI): the DDP bucket size (SURVEY.md §5.8 design rule 2: 25 -> 256 MB) and the
# gradient-reduction dtype at N = 2, 4, 8, the FSDP all-gather prefetch depth (1-3) and
# reduce-scatter dtype at N = 8, then the pipeline recipes' boundary (p2p) dtype and the PP x DP
# stage all-reduce dtype at N = 8, and the RCCL channel count against the GEMMs it shares CUs
# with (a 16-CU collective-sized occupier cost DDP 3.6 % on one GPU,
# profiles/r4_corun/; fewer channels = fewer co-resident CUs, at a lower ring bandwidth), and the
# peer-access transport (--comm ipc) and the N > 1 step graph against the RCCL defaults.  One
# JSON line per run in gpurun_out/scaling_sweep.jsonl.
#   bash scripts/scaling_sweep.sh [max_gpus]
set -u
MAXG=${1:-8}
OUT=gpurun_out/scaling_sweep.jsonl
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
port=29650
run() {  # $1 = N, rest = bench args
  local n=$1; shift
  port=$((port + 1))
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus "$n" --steps 10 --warmup 3 "$@" --json gpurun_out/_last.json > /dev/null 2>&1 || return $?
  python3 -c "import json,os,sys; d=json.load(open('gpurun_out/_last.json')); d['args']=sys.argv[1:]; d['nccl_channels']=os.environ.get('NCCL_MAX_NCHANNELS', ''); print(json.dumps(d))" "$@" >> $OUT
}
for n in 2 4 8; do
  [ "$n" -gt "$MAXG" ] && break
  for mb in 32 64 128 256; do
    for dt in fp32 bf16; do
      run $n --bucket_mb $mb --reduce_dtype $dt || exit $?
    done
  done
done
for pf in 1 2 3; do run "$MAXG" --recipe fsdp --prefetch $pf || exit $?; done  # FSDP all-gather depth
for dt in fp32 bf16; do run "$MAXG" --recipe fsdp --reduce_dtype $dt || exit $?; done  # FSDP RS dtype
for r in pipe pipe_ddp; do
  for w in fp32 bf16; do run "$MAXG" --recipe $r --pp_comm_dtype $w || exit $?; done  # PP wire dtype
done
for dt in fp32 bf16; do run "$MAXG" --recipe pipe_ddp --reduce_dtype $dt || exit $?; done  # PP x DP AR dtype
for n in 2 4 8; do  # the peer-access transport (parallel/ipc_comm.py: two-shot over all links) vs RCCL
  [ "$n" -gt "$MAXG" ] && break
  run $n --comm ipc || exit $?
  run $n --comm ipc --graph || exit $?
done
run "$MAXG" --recipe fsdp --comm ipc || exit $?
run "$MAXG" --graph || exit $?  # RCCL inside the captured step at N > 1
for ch in 4 8 16 32; do  # RCCL channels (CUs a collective occupies) under the DDP / FSDP steps
  NCCL_MIN_NCHANNELS=$ch NCCL_MAX_NCHANNELS=$ch run "$MAXG" || exit $?
  NCCL_MIN_NCHANNELS=$ch NCCL_MAX_NCHANNELS=$ch run "$MAXG" --recipe fsdp || exit $?
done
python3 - <<'PY'
import json
for l in open("gpurun_out/scaling_sweep.jsonl"):
    d = json.loads(l)
    print(d["n_gpus"], d["config"]["recipe"], " ".join(d["args"]), d.get("nccl_channels", ""), round(d["value"]), "tok/s")
PY
