#!/bin/bash
# v9 on / off for the plain nt products: the default bench alternated 4 times, same box.
for rep in 1 2 3 4; do
  scripts/gpu_step.sh "200:on_$rep:python -u bench.py" "200:off_$rep:DPC_G9=0 python -u bench.py" || exit $?
done
for rep in 1 2 3 4; do for v in on off; do echo -n "$v $rep: "; grep -o '"value": [0-9.]*' gpurun_out/${v}_$rep.log; done; done
