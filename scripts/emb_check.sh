#!/bin/bash
# Deterministic embedding backward: numerics / determinism tests, the HIP-graph and engine tests
# that run it inside captured steps, then DDP bench with the atomic scatter vs the sorted path.
scripts/gpu_step.sh \
  "300:t_emb:python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_engines_gpu.py -x -q --timeout 120 --timeout-method thread -k 'embedding or graph or engine or step'" \
  "150:b_atomic:env DPC_EMB_ATOMIC=1 python -u bench.py" \
  "150:b_sorted:python -u bench.py" \
  "150:b_atomic2:env DPC_EMB_ATOMIC=1 python -u bench.py" \
  "150:b_sorted2:python -u bench.py" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_emb -o e -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_emb.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
db=$(find gpurun_out/prof_emb -name "*.db" | head -1)
python3 scripts/kstats.py $db "emb" --top 40 | grep -E "eb_|emb_|radix|onesweep|rocprim|kstats|total" > gpurun_out/emb_kstats.txt
rm -rf gpurun_out/prof_emb
cat gpurun_out/emb_kstats.txt
