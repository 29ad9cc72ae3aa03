#!/bin/bash
# round 5 job 12: kernel table + PMC (MFMA busy, VALU/MFMA, clock) of the DDP step
set -o pipefail
R=$GRAFT_REPO_ROOT
scripts/gpu_step.sh "400:r5_prof12:scripts/prof_bench.sh r5b" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_r5b -o p -- python3 $R/bench.py --steps 2 --warmup 1 --no_graph > $R/gpurun_out/pmc_r5b.log 2>&1
rc=$?
cd $R
echo "pmc rc=$rc"; tail -2 gpurun_out/pmc_r5b.log
db=$(find gpurun_out/pmc_r5b -name "*.db" | head -1)
[ -n "$db" ] && python3 scripts/pmc_step.py $db "DDP step PMC, round 5 mid" > gpurun_out/pmc_r5b.md && cat gpurun_out/pmc_r5b.md
rm -rf gpurun_out/pmc_r5b
head -30 gpurun_out/prof_r5b_kstats.md
