#!/bin/bash
# Re-time the plain-product table entries, check every table signature's numerics with the new
# table, and A/B the DDP bench (new table vs the committed one), alternating processes.
NEW="DPC_GEMM_TABLE_PATH=gpurun_out/tuned_plain.json"
scripts/gpu_step.sh \
  "800:retune_plain:python -u bench/retune_keys.py --match ':00:a?\$' --impls 0 16 20 21 22 25 26 --write gpurun_out/tuned_plain.json" || exit $?
[ -f gpurun_out/tuned_plain.json ] || exit 3
scripts/gpu_step.sh \
  "300:sig_tests:env $NEW python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k table_signature" \
  "150:pab_new1:env $NEW python -u bench.py" "150:pab_old1:python -u bench.py" \
  "150:pab_new2:env $NEW python -u bench.py" "150:pab_old2:python -u bench.py"
