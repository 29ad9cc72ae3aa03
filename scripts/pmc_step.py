"""Per-kernel PMC table of one profiled training step (rocprofv3 --pmc database).

    python scripts/pmc_step.py gpurun_out/pmc_ddp/p_results.db "title" [--top 20]

Columns: dispatches, mean wall (us), effective clock (GRBM_GUI_ACTIVE / 8 XCDs / wall), MFMA
busy = SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024 SIMDs), VALU instructions per MFMA.
When the pass holds SQ_WAVE_CYCLES, two more columns: the share of wave cycles spent waiting on
any counter (SQ_WAIT_ANY, mostly vmcnt / lgkmcnt) and waiting for instruction issue
(SQ_WAIT_INST_ANY). Columns whose counters are absent from the pass print "-".
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
    mfma = (c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024)
            if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in c else None)
    vpm = (c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"]
           if c.get("SQ_INSTS_MFMA") and "SQ_INSTS_VALU" in c else None)
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    wait = c["SQ_WAIT_ANY"] / wc if wc and "SQ_WAIT_ANY" in c else None
    iwait = c["SQ_WAIT_INST_ANY"] / wc if wc and "SQ_WAIT_INST_ANY" in c else None
    rows.append((wall_ns, name, n, clock, mfma, vpm, wait, iwait))
rows.sort(reverse=True)
total = sum(r[0] for r in rows)
print(f"# {title}\n")


def pct(v):
    return "-" if v is None else f"{100 * v:.0f} %"


print("| kernel | calls | mean us | % time | clock GHz | MFMA busy | VALU / MFMA | wait any | wait inst |")
print("|---|---|---|---|---|---|---|---|---|")
for wall, name, n, clock, mfma, vpm, wait, iwait in rows[:top]:
    nm = name if len(name) < 90 else name[:87] + "..."
    v = "-" if vpm is None else f"{vpm:.1f}"
    print(f"| `{nm}` | {n} | {wall / n / 1e3:.1f} | {100 * wall / total:.1f} | {clock:.2f} | "
          f"{pct(mfma)} | {v} | {pct(wait)} | {pct(iwait)} |")
