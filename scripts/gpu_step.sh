#!/bin/bash
# Run GPU steps in order, each under its own time limit, stopping at the first step that
# crashed, faulted or timed out (exit codes other than 0/1).  Usage:
#   scripts/gpu_step.sh "<secs>:<name>:<command>" ["<secs>:<name>:<command>" ...]
# Each step's output goes to gpurun_out/<name>.log.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  secs="${spec%%:*}"; rest="${spec#*:}"
  name="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping: step $name ended with rc=$rc"
    exit $rc
  fi
done
exit 0
