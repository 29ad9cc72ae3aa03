"""Render rocprofv3 ``--kernel-trace --stats`` results as a markdown kernel table.

Reads either the CSV (``*_kernel_stats.csv``) or the rocpd SQLite database
(``*_results.db``, rocprofv3's default output) and prints the top kernels by total time.

    python scripts/kstats.py gpurun_out/prof/b_results.db "title" [--top 25] > profiles/x.md
"""
import csv
import sqlite3
import sys

path, title = sys.argv[1], sys.argv[2]
top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25
if path.endswith(".db"):
    con = sqlite3.connect(path)
    # per-kernel (name, calls, total ns)
    rows = [(n, c, t) for n, c, t in con.execute(
        "select name, count(*), sum(duration) from kernels group by name")]
else:
    rows = [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(path))]
rows.sort(key=lambda r: -r[2])
total = sum(r[2] for r in rows)
print(f"# {title}\n")
print(f"total kernel time {total / 1e6:.2f} ms over {sum(r[1] for r in rows)} launches\n")
print("| kernel | calls | total ms | avg us | % |")
print("|---|---|---|---|---|")
for name, calls, t in rows[:top]:
    name = name if len(name) < 110 else name[:107] + "..."
    print(f"| `{name}` | {calls} | {t / 1e6:.2f} | {t / calls / 1e3:.1f} | {100 * t / total:.2f} |")
