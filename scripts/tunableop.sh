#!/bin/bash
# hipBLASLt / rocBLAS solution tuning of the plain (epilogue-free) products through PyTorch
# TunableOp over the DDP bench (the GPT-2 XL / large shapes tune silently for minutes, longer
# than gpurun's output watchdog allows), merged into gpurun_out/hipblaslt_tuned.csv (copy it to
# distributed_pytorch_cookbook_amd/ops/); then A/B the DDP step with / without the table.
cp bench/hipblaslt_tuned.csv gpurun_out/hipblaslt_tuned.csv
T="PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/hipblaslt_tuned.csv"
scripts/gpu_step.sh "500:tune_ddp:$T python -u bench.py --steps 1 --warmup 1" || exit $?
scripts/gpu_step.sh "150:ab_off:DPC_TUNABLEOP=0 python -u bench.py" "150:ab_on:python -u bench.py" \
  "150:ab_off2:DPC_TUNABLEOP=0 python -u bench.py" "150:ab_on2:python -u bench.py"
