#!/bin/bash
# round 6 job 32: user-facing options end to end on the GPU (reference CLI defaults, 16 steps
# each): generation, f32 (--disable_amp), dropout + graph, recompute, grad scaler, FSDP CPU offload,
# the debug switches, save + resume
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
A="--synthetic_data --epochs 1 --max_steps 16 --num_workers 0"
run() {
  local name=$1; shift
  timeout -k 10 240 python -u "$@" > gpurun_out/r6_opt_$name.log 2>&1
  local rc=$?
  local last=$(tr '\r' '\n' < gpurun_out/r6_opt_$name.log | grep -E "\[training\]" | grep -v "?????" | tail -1 | sed 's/|[^|]*it\/s\]//' | cut -c1-110)
  local val=$(grep -E "^\[validation\]" gpurun_out/r6_opt_$name.log | tail -1)
  echo "$name rc=$rc | $last | $val"
  return $rc
}
run single_generate main-single.py $A --no_save || exit $?
grep -A4 "Argmax sampling" gpurun_out/r6_opt_single_generate.log | head -5
run disable_amp main-single.py $A --no_save --no_generate --disable_amp || exit $?
run dropout_graph main-single.py $A --no_save --no_generate --dropout 0.1 || exit $?
run recompute main-single.py $A --no_save --no_generate --recompute || exit $?
run grad_scaler main-single.py $A --no_save --no_generate --grad_scaler || exit $?
run fsdp_offload main-fsdp.py $A --no_save --no_generate --cpu_offload || exit $?
run stream_check main-ddp.py $A --no_save --no_generate --stream_check || exit $?
run serialize main-single.py $A --no_save --no_generate --serialize_kernels --max_steps 8 || exit $?
run save main-single.py $A --no_generate --checkpoint_dir gpurun_out/ck32 --save_every 8 || exit $?
run resume main-single.py --synthetic_data --epochs 1 --max_steps 24 --num_workers 0 --no_generate \
  --checkpoint_dir gpurun_out/ck32 --resume latest || exit $?
grep "\[resume\]" gpurun_out/r6_opt_resume.log
rm -rf gpurun_out/ck32
