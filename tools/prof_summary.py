"""Per-kernel summary of a rocprofv3 rocpd database (kernel trace).

usage: python tools/prof_summary.py run_results.db [csv_out]
"""
import sqlite3, sys, collections

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name_col = "kernel_name" if "kernel_name" in cols else "name"
rows = db.execute(f"select {name_col}, start, end from kernels order by start").fetchall()
agg = collections.OrderedDict()
for n, s, e in rows:
    n = n.split("(")[0]
    a = agg.setdefault(n, [0, 0.0, float("inf"), 0.0])
    d = (e - s) / 1e6
    a[0] += 1; a[1] += d; a[2] = min(a[2], d); a[3] = max(a[3], d)
tot = sum(a[1] for a in agg.values())
lines = ["Name,Calls,TotalDurationMs,AverageMs,MinMs,MaxMs,Percentage"]
for n, a in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    lines.append(f"{n},{a[0]},{a[1]:.4f},{a[1]/a[0]:.5f},{a[2]:.5f},{a[3]:.5f},{100*a[1]/tot:.2f}")
out = "\n".join(lines)
print(out)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(out + "\n")
