#!/bin/bash
# round 6 job 14: peer-access collectives at 256 workgroups: their tests, the microbench, the N = 2
# one-GPU graph rehearsal of bench.py (now reporting comm / step_graph), then every GPU test
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/jobs/r6_job12.sh || exit $?
scripts/jobs/r6_job13.sh || exit $?
scripts/gpu_step.sh "600:r6_gputests14:python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" || exit $?
