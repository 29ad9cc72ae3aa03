"""Per-step GPU busy time vs wall time from a rocprofv3 kernel trace (rocpd SQLite DB).

Steps are delimited by the AdamW kernel (the last kernel of every training step).  For the
last ``--steps`` steps it prints, per step, the wall time between consecutive AdamW ends,
the union of kernel intervals inside it (GPU busy) and the idle gap, then the mean, and the
per-kernel time of one mean step.

    python scripts/step_gaps.py gpurun_out/prof/b_results.db [--steps 8] [--delim adamw] [--seq out.txt]

--seq writes the last step's dispatches in launch order (duration, grid, name) to a file: the
per-call view (which GEMM shape costs what) that the per-kernel totals hide.
"""
import sqlite3
import sys
from collections import defaultdict

path = sys.argv[1]
nsteps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 8
delim = sys.argv[sys.argv.index("--delim") + 1] if "--delim" in sys.argv else "adamw"
con = sqlite3.connect(path)
cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
s_col = "start" if "start" in cols else ("begin" if "begin" in cols else None)
e_col = "end" if "end" in cols else None
if s_col is None or e_col is None:
    sys.exit(f"unexpected kernels columns: {cols}")
rows = sorted(con.execute(f'select name, "{s_col}", "{e_col}" from kernels'), key=lambda r: r[1])
ends = [e for n, s, e in rows if delim in n]
if len(ends) < nsteps + 1:
    sys.exit(f"only {len(ends)} '{delim}' kernels")
# an AdamW may be split into several launches per step (DDP buckets): keep the last of a burst
marks = []
for e in ends:
    if marks and e - marks[-1] < 2e6:  # < 2 ms apart: same step
        marks[-1] = e
    else:
        marks.append(e)
if len(marks) < nsteps + 1:  # (fewer steps traced than asked: use what there is)
    print(f"(only {len(marks) - 1} step boundaries found; using them)")
    nsteps = len(marks) - 1
marks = marks[-(nsteps + 1):]
per_kernel = defaultdict(float)
tot_wall = tot_busy = 0.0
for i in range(nsteps):
    lo, hi = marks[i], marks[i + 1]
    iv = [(max(s, lo), min(e, hi), n) for n, s, e in rows if e > lo and s < hi]
    busy, cur_s, cur_e = 0.0, None, None
    for s, e, n in sorted(iv):
        per_kernel[n] += (e - s) / nsteps
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    wall = hi - lo
    tot_wall += wall
    tot_busy += busy
    print(f"step {i}: wall {wall / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(wall - busy) / 1e6:.3f} ms")
print(f"mean: wall {tot_wall / nsteps / 1e6:.3f} ms  busy {tot_busy / nsteps / 1e6:.3f} ms  "
      f"idle {(tot_wall - tot_busy) / nsteps / 1e6:.3f} ms")
if "--seq" in sys.argv:
    lo, hi = marks[-2], marks[-1]
    gcol = [c for c in cols if c in ("grid_size", "grid_x", "grid_size_x", "workgroup_count")]
    sel = f'select name, "{s_col}", "{e_col}"' + (f', "{gcol[0]}"' if gcol else "") + " from kernels"
    seq = sorted((r for r in con.execute(sel) if r[2] > lo and r[1] < hi), key=lambda r: r[1])
    with open(sys.argv[sys.argv.index("--seq") + 1], "w") as f:
        f.write(f"# columns: {cols}\n")
        for r in seq:
            g = r[3] if gcol else ""
            f.write(f"{(r[2] - r[1]) / 1e3:9.1f} us  {g}  {r[0][:110]}\n")
print("\n| kernel | ms per step |\n|---|---|")
for n, t in sorted(per_kernel.items(), key=lambda kv: -kv[1])[:30]:
    n = n if len(n) < 100 else n[:97] + "..."
    print(f"| `{n}` | {t / 1e6:.3f} |")
