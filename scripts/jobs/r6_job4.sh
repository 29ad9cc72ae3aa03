#!/bin/bash
# round 6 job 4: stock PyTorch-ROCm yardsticks for the FSDP XL / pipe medium / PP x DP large configs
# at N = 1, 64 sequences per GPU: the reference math (manual
# attention) + torch.compile with gradient accumulation where one 64-sequence batch of scores does
# not fit, SDPA + compile on the whole batch, and torch FSDP-wrapped for XL
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
(while sleep 45; do date >> gpurun_out/r6_hb.txt; done) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
out=gpurun_out/r6_stock.jsonl
: > $out
run() {  # <limit> <args...>
  local lim=$1; shift
  echo "== stock $*"
  timeout -k 10 $lim python -u bench/baseline_torch.py --steps 5 --warmup 3 "$@" > gpurun_out/r6_stock_last.log 2>&1
  local rc=$?
  grep '^{' gpurun_out/r6_stock_last.log | tee -a $out
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r6_stock_last.log; }
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
run 500 --model gpt2-medium --batch_size 64 --sdpa --compile
run 500 --model gpt2-medium --batch_size 16 --accum 4 --compile
run 600 --model gpt2-large --batch_size 64 --sdpa --compile
run 600 --model gpt2-large --batch_size 16 --accum 4 --compile
run 700 --model gpt2-xl --batch_size 64 --sdpa --compile
run 700 --model gpt2-xl --batch_size 8 --accum 8 --compile
run 700 --model gpt2-xl --batch_size 64 --sdpa --compile --fsdp
