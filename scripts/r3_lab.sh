#!/bin/bash
# bench/g7lab runs (GEMM schedule A/B + ablations); args: one "name:M N K layout rounds reps set" per step
specs=()
for a in "$@"; do
  name="${a%%:*}"; rest="${a#*:}"
  specs+=("120:$name:bench/g7lab $rest")
done
scripts/gpu_step.sh "${specs[@]}"
