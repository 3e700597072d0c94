"""Per-kernel L2 hit rate from one rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum pass.

python tools/pmc_l2.py <counter_collection.csv> [top]
Rows: kernel (name + grid), launches, average hits and misses per launch (64-B requests, all channels), hit
rate, and the miss bytes per launch (misses x 128 B: the L2 line a miss fills from the fabric)."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for r in csv.DictReader(open(path)):
    grid = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
    key = (r["Kernel_Name"][:90], grid)
    acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[key].add(r["Dispatch_Id"])
rows = []
for key, c in acc.items():
    n = len(disp[key])
    hit, miss = c.get("TCC_HIT_sum", 0.0) / n, c.get("TCC_MISS_sum", 0.0) / n
    rows.append((hit + miss, key, n, hit, miss))
rows.sort(reverse=True)
for tot, (name, grid), n, hit, miss in rows[:top]:
    rate = hit / tot if tot else 0.0
    print(f"{name:90s} grid={grid:6d} n={n:3d} hit={hit / 1e6:8.2f}M miss={miss / 1e6:7.2f}M rate={rate:6.3f} "
          f"miss_MB={miss * 128 / 1e6:8.1f}")
