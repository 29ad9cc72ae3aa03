#!/bin/bash
# round 5 job 62: a longer DDP run (200 timed steps) on the final kernels -- the loss stays finite
# and the step time stable -- and 20 FSDP XL steps
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 200 --warmup 5 2>&1 | grep -v amdgpu.ids | cut -c1-400 || exit 1
timeout -k 10 300 python -u bench.py --recipe fsdp --steps 20 --warmup 3 2>&1 | grep -v amdgpu.ids | cut -c1-400 || exit 1
