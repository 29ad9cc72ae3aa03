#!/bin/bash
# round 5 job 64: multi-rank rehearsal (gloo ranks sharing the one MI355X, real kernels) on the final tree
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/rehearse_multirank.sh 3 || exit $?
