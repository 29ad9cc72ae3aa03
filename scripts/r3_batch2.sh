#!/bin/bash
# Round-3 batch 2: the paired-M0 DMA schedule as the default -- every GPU test, the four
# recipe benches, the LDS-occupier reserve measurement, kernel tables of the forced N > 1 paths.
scripts/gpu_step.sh "400:gputests:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "150:b_ddp:python -u bench.py" \
  "150:b_ddp_nopair:env DPC_G7_PAIR=0 python -u bench.py" \
  "150:b_ddp2:python -u bench.py" \
  "200:b_fsdp:python -u bench.py --recipe fsdp --steps 8 --warmup 3" \
  "200:b_pipe:python -u bench.py --recipe pipe --steps 8 --warmup 3" \
  "200:b_ppd:python -u bench.py --recipe pipe_ddp --steps 8 --warmup 3" \
  "200:cu_reserve_lds:python -u bench/cu_reserve.py" || exit $?
bash scripts/prof_bench.sh fd_fsdp --recipe fsdp --force_dist_path && \
bash scripts/prof_bench.sh base_fsdp --recipe fsdp && \
bash scripts/prof_bench.sh fd_ddp --force_dist_path && \
bash scripts/prof_bench.sh base_ddp
