"""Per-kernel averages of rocprofv3 --pmc counters over one or more passes (one counter set per pass).

python tools/pmc_kernels.py <counter_collection.csv> [<counter_collection.csv> ...]
Rows: kernel (short name + grid), launches, the mean per launch of every counter the passes hold, and where the
counters are present: HBM read MB (FETCH_SIZE x 2: the gfx950 correction of MI355X_MICROARCH.md's HBM section),
write MB (WRITE_SIZE), L2 hit rate (TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)) and the MFMA-busy fraction
(SQ_VALU_MFMA_BUSY_CYCLES summed over the 1,024 SIMDs, per kernel cycle = GRBM_GUI_ACTIVE / 8).  Vendor (Cijk) kernels are named by
their macro tile, wave tile and stream-K tokens."""
import csv
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    if "Cijk" in name:
        mt = re.search(r"MT\d+x\d+x\d+", name)
        wt = re.search(r"MIWT\d+_\d+", name)
        return "vendor " + " ".join(x for x in (mt.group(0) if mt else "?", wt.group(0) if wt else "",
                                                  "SK3" if "SK3" in name else "") if x)
    n = name.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    return "engine " + n.split("(")[0][:70]


acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(lambda: defaultdict(set))
order = []
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        grid = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
        key = (short(r["Kernel_Name"]), grid)
        if key not in acc:
            order.append(key)
        acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[key][r["Counter_Name"]].add((path, r["Dispatch_Id"]))
for key in order:
    c = acc[key]
    mean = {k: v / max(1, len(disp[key][k])) for k, v in c.items()}
    n = max(len(s) for s in disp[key].values())
    parts = []
    if "FETCH_SIZE" in mean:
        parts.append(f"read={mean['FETCH_SIZE'] * 2 / 1e3:8.1f}MB")  # FETCH_SIZE is in KB
    if "WRITE_SIZE" in mean:
        parts.append(f"write={mean['WRITE_SIZE'] / 1e3:7.1f}MB")
    if "TCC_HIT_sum" in mean and "TCC_MISS_sum" in mean:
        tot = mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"]
        parts.append(f"l2hit={mean['TCC_HIT_sum'] / tot if tot else 0:.3f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in mean and mean.get("GRBM_GUI_ACTIVE"):
        # MFMA-busy cycles summed over the 1,024 SIMDs / the kernel's cycles (GRBM_GUI_ACTIVE sums the 8 XCDs)
        cyc = mean["GRBM_GUI_ACTIVE"] / 8
        parts.append(f"mfma_busy={mean['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / cyc:.3f} cycles={cyc:.0f}")
    rest = " ".join(f"{k}={v:.4g}" for k, v in sorted(mean.items())
                    if k not in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"))
    print(f"{key[0]:72s} grid={key[1]:5d} n={n:3d} {' '.join(parts)} {rest}")
