"""Summarise a rocprofv3 kernel profile per bench step.

python tools/prof_summary.py <kernel_stats.csv | results.db> <steps> [top]
For a rocpd SQLite database (rocprofv3's default output) kernels are also split by grid size,
which separates e.g. the stage-1 and cross-attention launches of one kernel."""
import csv
import sqlite3
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
if path.endswith(".db"):
    c = sqlite3.connect(path)
    rows = {}
    for name, gx, gy, gz, wx, dur in c.execute(
            "select name, grid_x, grid_y, grid_z, workgroup_x, duration from kernels"):
        key = (name, f"{gx // max(wx, 1)}x{gy}x{gz}")
        r = rows.setdefault(key, [0, 0.0])
        r[0] += 1
        r[1] += float(dur)
    tot = sum(v[1] for v in rows.values())
    for (name, grid), (calls, ns) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{ns/1e6/steps:8.3f} ms/step {100*ns/tot:6.2f}% calls/step={calls/steps:6.1f} "
              f"avg={ns/calls/1e3:9.1f}us grid={grid:12s} {name[:90]}")
else:
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step {float(r['Percentage']):6.2f}% "
              f"calls/step={int(r['Calls'])/steps:6.1f} avg={float(r['AverageNs'])/1e3:9.1f}us  {r['Name'][:96]}")
print(f"total {tot/1e6/steps:.3f} ms/step")
