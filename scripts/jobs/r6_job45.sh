#!/bin/bash
# round 6 job 45: the dQ kernel with both 32-key sub-blocks' S / dP MFMAs issued first (four
# independent chains; DPC_ATTN_VAR bwd 5) against the shipped one (bwd 1): bitwise equality, the
# attention tests on variant 5, then interleaved timings at the GPT-2 small step shape
mkdir -p gpurun_out
set -o pipefail
O=gpurun_out/r6_dqilp
mkdir -p $O
DPC_ATTN_VAR=9,1 timeout -k 10 120 python -u scripts/jobs/attn_dump.py $O/v1.pt > $O/dump1.log 2>&1 &&
DPC_ATTN_VAR=9,5 timeout -k 10 120 python -u scripts/jobs/attn_dump.py $O/v5.pt > $O/dump5.log 2>&1 &&
python -c "
import torch; a=torch.load('$O/v1.pt'); b=torch.load('$O/v5.pt')
print('bitwise equal:', torch.equal(a, b), 'max abs diff', (a.float()-b.float()).abs().max().item())" | tee $O/eq.txt &&
rm -f $O/*.pt &&
DPC_ATTN_VAR=9,5 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k attention -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $O/tests_v5.log 2>&1 && tail -1 $O/tests_v5.log &&
for v in 1 5 1 5; do
  DPC_ATTN_VAR=9,$v timeout -k 10 120 python -u bench/attn_time.py >> $O/time.log 2>&1 || exit 1
  echo "var $v: $(tail -1 $O/time.log)"
done
