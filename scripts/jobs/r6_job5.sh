#!/bin/bash
# round 6 job 5: the round-end check on this tree -- every GPU test, smoke, the four recipe benches,
# the zero-bubble stage proxy (zb2 order executed), and two PMC passes over the DDP step
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_step.sh "600:r6_gputests:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "120:r6_smoke:python -u __graft_entry__.py" \
  "150:r6_b_ddp:python -u bench.py" \
  "300:r6_b_fsdp:python -u bench.py --recipe fsdp --steps 8 --warmup 3" \
  "200:r6_b_pipe:python -u bench.py --recipe pipe --steps 8 --warmup 3" \
  "300:r6_b_ppd:python -u bench.py --recipe pipe_ddp --steps 8 --warmup 3" || exit $?
for args in "--model gpt2-medium --pp 8 --micro 16 --mb 32" "--model gpt2-large --pp 2 --micro 4 --mb 32"; do
  timeout -k 10 300 python -u bench/pp_stage_proxy.py $args --schedule zb2 --steps 3 --warmup 1 \
    >> gpurun_out/r6_proxy_zb2.jsonl 2> gpurun_out/r6_proxy_err.log || { tail -5 gpurun_out/r6_proxy_err.log; exit 4; }
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE \
  -d $R/gpurun_out/pmc5a -o p -- python3 $R/bench.py --steps 2 --warmup 1 --no_graph > $R/gpurun_out/pmc5a.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
  -d $R/gpurun_out/pmc5b -o p -- python3 $R/bench.py --steps 2 --warmup 1 --no_graph > $R/gpurun_out/pmc5b.log 2>&1
rc=$?
cd $R
a=$(find gpurun_out/pmc5a -name '*.db' | head -1); b=$(find gpurun_out/pmc5b -name '*.db' | head -1)
[ -n "$a" ] && python3 scripts/pmc_step.py $a "pass A" > gpurun_out/r6_pmc_a.md
[ -n "$b" ] && python3 scripts/pmc_step.py $b "pass B" > gpurun_out/r6_pmc_b.md
rm -rf gpurun_out/pmc5a gpurun_out/pmc5b
exit $rc
