"""Stage-1 vs cross-attention launches of the stream-K attention kernel in a rocprofv3 SQLite result (both run
attn_sk_kernel on a 256-workgroup grid, so a per-name/grid summary merges them).  Each frame launches the kernel
14 times for stage 1, then 10 times for the decoder's cross-attention (large-proxy, one view): launches are taken in
start order and split 14 / 10 per frame; the stage-1 average is what bench.py's roofline times.

python tools/attn_split.py <run_results.db> [stage1_layers=14] [cross_layers=10]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
l1 = int(sys.argv[2]) if len(sys.argv) > 2 else 14
l2 = int(sys.argv[3]) if len(sys.argv) > 3 else 10
d = [r[0] / 1000.0 for r in c.execute("select duration from kernels where name like '%attn_sk_kernel%' "
                                       "order by start")]
per = l1 + l2
frames = len(d) // per
s1 = [x for f in range(frames) for x in d[f * per:f * per + l1]]
s2 = [x for f in range(frames) for x in d[f * per + l1:(f + 1) * per]]
print(f"attn_sk_kernel launches {len(d)} = {frames} frames x ({l1} stage-1 + {l2} cross)")
print(f"stage-1: n={len(s1)} avg={sum(s1) / max(1, len(s1)):.1f} us  min={min(s1):.1f}  max={max(s1):.1f}")
print(f"cross:   n={len(s2)} avg={sum(s2) / max(1, len(s2)):.1f} us  min={min(s2):.1f}  max={max(s2):.1f}")
