#!/bin/bash
# hipBLASLt's kernel choice (name, grid, workgroup, LDS, VGPR) for the GPT-2-small products
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/blasprobe -o b -- python3 $R/bench/blas_probe.py > $R/gpurun_out/blasprobe.log 2>&1
cd $R
f=$(find gpurun_out/blasprobe -name "*kernel_trace.csv" | head -1)
python3 - "$f" > gpurun_out/blasprobe_kernels.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
print(list(rows[0].keys()))
seen = collections.OrderedDict()
for r in rows:
    k = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    seen.setdefault(k, []).append((d, r))
for k, v in seen.items():
    d, r = v[-1]
    print(f"{d:9.1f} us  grid {r.get('Grid_Size_X')}x{r.get('Grid_Size_Y')}x{r.get('Grid_Size_Z')} wg {r.get('Workgroup_Size_X')} "
          f"lds {r.get('Group_Segment_Size', r.get('LDS_Block_Size'))} vgpr {r.get('Arch_VGPR_Count', r.get('VGPR_Count'))} "
          f"agpr {r.get('Accum_VGPR_Count')} sgpr {r.get('SGPR_Count')} n={len(v)}\n    {k[:300]}")
PY
rm -rf gpurun_out/blasprobe
cat gpurun_out/blasprobe_kernels.txt
