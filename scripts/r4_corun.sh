#!/bin/bash
# CU co-residency of the multi-GPU steps on one MI355X: the engines' N > 1 code path at one rank
# (--force_dist_path) with every collective followed by a collective-sized occupier on the comm
# stream (DPC_FAKE_COLL = CUs, bus GB/s, world), against the resident-CU reserve of the
# persistent GEMMs (DPC_CU_RESERVE)
for cus in 16 32; do
  for res in 0 16 32; do
    scripts/gpu_step.sh "150:co_ddp_c${cus}_r${res}:DPC_FAKE_COLL=$cus,300,8 DPC_CU_RESERVE=$res python -u bench.py --force_dist_path" || exit $?
  done
done
scripts/gpu_step.sh "150:co_ddp_nofake:python -u bench.py --force_dist_path" || exit $?
for res in 0 16 32; do
  scripts/gpu_step.sh "200:co_fsdp_c16_r${res}:DPC_FAKE_COLL=16,300,8 DPC_CU_RESERVE=$res python -u bench.py --recipe fsdp --force_dist_path --steps 6 --warmup 2" || exit $?
done
scripts/gpu_step.sh "200:co_fsdp_nofake:python -u bench.py --recipe fsdp --force_dist_path --steps 6 --warmup 2" || exit $?
for f in gpurun_out/co_*.log; do
  echo "$f $(grep -h '"value"' $f | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
