"""Summarise a rocprofv3 PMC database: mean counter value per dispatch of kernels matching a pattern.

    python scripts/pmc_summary.py gpurun_out/pmc_x_a/p_results.db gemm
"""
import sqlite3
import sys
from collections import defaultdict

db, pat = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
agg = defaultdict(list)
dur = {}
for name, cnt, val, disp, d in c.execute(
        "select kernel_name, counter_name, value, dispatch_id, duration from counters_collection"):
    if pat in name:
        agg[cnt].append(val)
        dur[disp] = d
print(f"dispatches={len(dur)} mean_duration_us={sum(dur.values()) / max(len(dur), 1) / 1e3:.1f}")
for k in sorted(agg):
    v = agg[k]
    print(f"{k:36s} {sum(v) / len(v):16.1f}")
