#!/bin/bash
# round 5 job 6: EPI 8 column sums masked on rows past M; the whole GPU suite
scripts/gpu_step.sh \
  "900:r5_t6:python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu"
