"""Per-kernel PMC table of one profiled training step (rocprofv3 --pmc database).

    python scripts/pmc_step.py gpurun_out/pmc_ddp/p_results.db "title" [--top 20]

Columns: dispatches, mean wall (us), effective clock (GRBM_GUI_ACTIVE / 8 XCDs / wall), MFMA
busy = SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024 SIMDs), VALU instructions per MFMA.
"""
import sqlite3
import sys
from collections import defaultdict

db, title = sys.argv[1], sys.argv[2]
top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 20
con = sqlite3.connect(db)
vals = defaultdict(lambda: defaultdict(float))  # (kernel) -> counter -> sum over dispatches
disp = defaultdict(dict)  # kernel -> dispatch -> duration ns
for name, cnt, val, d, dur in con.execute(
        "select kernel_name, counter_name, value, dispatch_id, duration from counters_collection"):
    vals[name][cnt] += val
    disp[name][d] = dur
rows = []
for name, ds in disp.items():
    n = len(ds)
    wall_ns = sum(ds.values())
    c = vals[name]
    cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    clock = cyc / wall_ns if wall_ns else 0.0
    mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (cyc * 1024) if cyc else 0.0
    vpm = c.get("SQ_INSTS_VALU", 0.0) / c["SQ_INSTS_MFMA"] if c.get("SQ_INSTS_MFMA") else float("nan")
    rows.append((wall_ns, name, n, clock, mfma, vpm))
rows.sort(reverse=True)
total = sum(r[0] for r in rows)
print(f"# {title}\n")
print("| kernel | calls | mean us | % time | clock GHz | MFMA busy | VALU / MFMA |")
print("|---|---|---|---|---|---|---|")
for wall, name, n, clock, mfma, vpm in rows[:top]:
    nm = name if len(name) < 90 else name[:87] + "..."
    print(f"| `{nm}` | {n} | {wall / n / 1e3:.1f} | {100 * wall / total:.1f} | {clock:.2f} | {100 * mfma:.0f} % | {vpm:.1f} |")
