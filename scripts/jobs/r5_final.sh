#!/bin/bash
# round 5 final check: the driver's round-end steps (GPU tests, smoke, bench) plus the recipe
# benches and the DDP step's kernel table
scripts/round_check.sh || exit $?
scripts/gpu_step.sh "400:r5_prof_final:scripts/prof_bench.sh r5f"
