#!/bin/bash
# What the driver runs at round end, plus the four recipe benches, on one MI355X.
scripts/gpu_step.sh "400:gputests:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "120:smoke:python -u __graft_entry__.py" \
  "150:b_ddp:python -u bench.py" \
  "200:b_fsdp:python -u bench.py --recipe fsdp --steps 8 --warmup 3" \
  "200:b_pipe:python -u bench.py --recipe pipe --steps 8 --warmup 3" \
  "200:b_ppd:python -u bench.py --recipe pipe_ddp --steps 8 --warmup 3"
