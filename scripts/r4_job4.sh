#!/bin/bash
# same-box A/B: e66e941 (ab_old/) vs this tree (scalar alpha, ER 4 default) vs this tree with the
# up-projection forward on v9 (a table with every bias+GELU+aux_out forward key -> impl 26, made
# here; the shipped table has them since); FSDP old vs new; kernel profiles of the pipeline stage
# proxy (micro-batched vs one batch).  Results: profiles/r4_ab/, profiles/r4_pp/.
R=$PWD
mkdir -p gpurun_out
python3 - <<'PY'
import json
t = json.load(open("distributed_pytorch_cookbook_amd/ops/gemm_tuned.json"))
for k in t["impl"]:
    if k.endswith(":kk:h:20:bx"):
        t["impl"][k] = 26
json.dump(t, open("gpurun_out/gemm_tuned_g9fwd.json", "w"), indent=1, sort_keys=True)
PY
scripts/gpu_step.sh "300:warm:python -u scripts/warm.py" || exit $?
(cd ab_old && timeout -k 10 300 python -u ../scripts/warm.py > $R/gpurun_out/warm_old.log 2>&1) || exit $?
for rep in 1 2 3; do
  (cd ab_old && timeout -k 10 150 python -u bench.py > $R/gpurun_out/e_old_$rep.log 2>&1) || exit $?
  timeout -k 10 150 python -u bench.py > gpurun_out/e_new_$rep.log 2>&1 || exit $?
  DPC_GEMM_TABLE_PATH=gpurun_out/gemm_tuned_g9fwd.json timeout -k 10 150 python -u bench.py > gpurun_out/e_g9f_$rep.log 2>&1 || exit $?
  DPC_G9_ER=0 timeout -k 10 150 python -u bench.py > gpurun_out/e_er0_$rep.log 2>&1 || exit $?
done
for f in gpurun_out/e_*.log; do
  echo "$f $(grep -h '"value"' $f | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
(cd ab_old && timeout -k 10 200 python -u bench.py --recipe fsdp --steps 6 --warmup 2 > $R/gpurun_out/f_old.log 2>&1) || exit $?
DPC_GEMM_TABLE_PATH=gpurun_out/gemm_tuned_g9fwd.json timeout -k 10 200 python -u bench.py --recipe fsdp --steps 6 --warmup 2 > gpurun_out/f_g9f.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --recipe fsdp --steps 6 --warmup 2 > gpurun_out/f_new.log 2>&1 || exit $?
for f in gpurun_out/f_*.log; do
  echo "$f $(grep -h '"value"' $f | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ppm -o run -- python -u bench/pp_stage_proxy.py --model gpt2-medium --pp 8 --micro 32 --mb 16 --only micro --steps 3 --warmup 1 > gpurun_out/prof_ppm.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ppf -o run -- python -u bench/pp_stage_proxy.py --model gpt2-medium --pp 8 --micro 32 --mb 16 --only full --steps 3 --warmup 1 > gpurun_out/prof_ppf.log 2>&1 || exit $?
