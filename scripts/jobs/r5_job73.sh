#!/bin/bash
# round 5 job 73: two PMC passes over a short DDP bench step (no graph, so each kernel is its own
# dispatch): pass 1 MFMA busy / instruction mix, pass 2 wave-cycle wait shares
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE \
  -d $R/gpurun_out/pmc73a -o p -- python3 $R/bench.py --steps 2 --warmup 1 --no_graph \
  > $R/gpurun_out/pmc73a.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
  -d $R/gpurun_out/pmc73b -o p -- python3 $R/bench.py --steps 2 --warmup 1 --no_graph \
  > $R/gpurun_out/pmc73b.log 2>&1
rc=$?
find $R/gpurun_out/pmc73a $R/gpurun_out/pmc73b -name '*.db' 2>/dev/null
exit $rc
