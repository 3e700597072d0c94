"""Per-kernel duration stats from a rocprofv3 SQLite result (rocpd `kernels` view), in first-launch order.

python tools/rocpd_stats.py <run_results.db> [name-substring]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
pat = f"%{sys.argv[2]}%" if len(sys.argv) > 2 else "%"
rows = c.execute("select name, grid_x / workgroup_x, count(*), avg(duration) / 1000.0, min(duration) / 1000.0, "
                 "min(start) from kernels where name like ? group by name, grid_x order by min(start)", (pat,))
for name, grid, n, avg, mn, _ in rows:
    short = name.replace("(anonymous namespace)::", "").split("(")[0]
    print(f"{short[:70]:70s} grid={grid:6d} n={n:4d} avg={avg:9.1f}us min={mn:9.1f}us")
