"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> [out.json]

Corrections follow MI355X_MICROARCH.md §HBM: both counters are in KiB; on gfx950 FETCH_SIZE
tallies exactly half of the bytes of wide (16 B/lane) coalesced reads, so it is doubled; WRITE_SIZE
is exact for 16-B stores.  Rows are grouped by (kernel, grid size) so that e.g. the stage-1 and the
cross-attention launches of one kernel stay apart.  The stage-1 attention entry (grid of the
bench workload) is written to profiles/attn_stage1_traffic.json (or $RF_TRAFFIC_OUT) for bench.py's
roofline.traffic, with the digest of the attention sources it was measured on: bench.py reports the figure
only while the sources still match (run this on the GPU box right after the passes, tools/gpu.sh round)."""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from renderformer_amd._lib import ATTN_SOURCES, source_digest  # noqa: E402


ATTN_CYCLE = (14, 10)  # bench frame: 14 stage-1 then 10 cross-attention launches of attn_sk_kernel


def load(path, counter):
    """Average per (kernel, grid); the stream-K attention launches all have grid = #CUs, so they are split
    into stage-1 / cross by their position in the per-frame launch sequence."""
    per = defaultdict(list)
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    n_attn = 0
    for r in rows:
        name = r["Kernel_Name"]
        grid = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
        if "attn_sk_kernel" in name:
            name += " [stage-1]" if n_attn % sum(ATTN_CYCLE) < ATTN_CYCLE[0] else " [cross]"
            n_attn += 1
        per[(name, grid)].append(float(r["Counter_Value"]) * 1024.0)
    return per


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    rows = []
    for key in sorted(set(fetch) | set(write), key=lambda k: -sum(fetch.get(k, [0]))):
        f, w = fetch.get(key, []), write.get(key, [])
        fb = 2.0 * sum(f) / len(f) if f else float("nan")
        wb = sum(w) / len(w) if w else float("nan")
        rows.append({"kernel": key[0], "grid": key[1], "launches": len(f), "read_bytes_per_launch": fb,
                     "write_bytes_per_launch": wb, "hbm_bytes_per_launch": fb + wb})
    for r in rows[:25]:
        print(f"{r['hbm_bytes_per_launch']/1e6:10.2f} MB/launch (rd {r['read_bytes_per_launch']/1e6:9.2f} "
              f"wr {r['write_bytes_per_launch']/1e6:9.2f}) n={r['launches']:4d} grid={r['grid']:6d} {r['kernel'][:90]}")
    if len(sys.argv) > 3:
        json.dump(rows, open(sys.argv[3], "w"), indent=1)
    st1 = [r for r in rows if "[stage-1]" in r["kernel"]]
    if st1:
        json.dump({"kernel": st1[0]["kernel"], "hbm_bytes_per_launch": st1[0]["hbm_bytes_per_launch"],
                   "read_bytes_per_launch": st1[0]["read_bytes_per_launch"],
                   "write_bytes_per_launch": st1[0]["write_bytes_per_launch"], "launches": st1[0]["launches"],
                   "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --profile (separate runs)",
                   "source_digest": source_digest(*ATTN_SOURCES)},
                  open(os.environ.get("RF_TRAFFIC_OUT", "profiles/attn_stage1_traffic.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
