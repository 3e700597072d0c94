"""Average PMC counters per dispatch of one kernel: python tools/pmc_summary.py <dir> <kernel substring> [grid]"""
import csv
import glob
import sys
from collections import defaultdict

root, name = sys.argv[1], sys.argv[2]
grid = int(sys.argv[3]) if len(sys.argv) > 3 else None
vals = defaultdict(list)
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if name not in r["Kernel_Name"]:
            continue
        if grid is not None and int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"])) != grid:
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
