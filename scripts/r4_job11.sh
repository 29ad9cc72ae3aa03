#!/bin/bash
# PMC counters over three DDP steps: per-kernel effective clock, MFMA busy and VALU per MFMA
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 300 python -u scripts/warm.py > gpurun_out/warm.log 2>&1 || exit $?
cd /tmp && timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
  -d $R/gpurun_out/pmc_ddp -o p -- python3 $R/bench.py --steps 2 --warmup 1 --no_graph > $R/gpurun_out/pmc_ddp.log 2>&1 || exit $?
cd $R && python3 scripts/pmc_step.py $(find gpurun_out/pmc_ddp -name "*.db" | head -1) "GPT-2 small DDP, 3 steps under PMC" --top 20
