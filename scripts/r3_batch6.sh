#!/bin/bash
# Full GPU suite on the reverted-epilogue tree, then the --cpu_offload stage breakdown.
scripts/gpu_step.sh "400:gputests:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200:off_none:python -u bench/offload.py --offload 0" \
  "300:off_break:python -u bench/offload.py --breakdown"
