"""Stage-1 stream-K attention at the bench shape under the RF_ATTN_DBG ablation builds (timing only).

python tools/attn_ablate.py            -> one line per variant
python tools/attn_ablate.py pmc [reps] -> just the shipped kernel, `reps` launches (for rocprofv3 --pmc)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from renderformer_amd import ops  # noqa: E402
from renderformer_amd._lib import load  # noqa: E402

load()
S, D, H = 5649, 1024, 8
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.randn(S, 3 * D, device="cuda", generator=g).bfloat16()
qs = (qkv[:, :D].float() * ops.Q_LOG2_SCALE).bfloat16()
out = torch.empty(S, D, device="cuda", dtype=torch.bfloat16)
prob = torch.tensor([[0, S, 0, S, 0]], dtype=torch.int32, device="cuda")


def run():
    ops.attention(qs, qkv[:, D:2 * D], qkv[:, 2 * D:], out, prob, S, H, q_prescaled=True)


if len(sys.argv) > 1 and sys.argv[1] == "stamps":
    os.environ["RF_ATTN_DBG"] = sys.argv[2] if len(sys.argv) > 2 else "32"
    for _ in range(30):
        run()
    torch.cuda.synchronize()
    ws = ops._attn_workspace(out.device)
    piece = (ws.numel() - 512) // 512
    st = ws[511 * piece:511 * piece + 256 * 8 * 16].view(torch.int64).view(256, 8, 8).cpu().double()
    tiles = st[..., 7].clamp_min(1)
    names = ["top wait", "A (+K DMA, check)", "seam wait", "B (+V DMA)"]
    clk = (st[..., 4] / st[..., 5].clamp_min(1)).median() * 100.0
    print(f"in-kernel shader clock (s_memtime / s_memrealtime x 100 MHz, median over waves): {clk:.0f} MHz")
    tot = st[..., 4].mean()
    loop = st[..., :4].sum(-1).mean()
    pro = st[..., 6].mean()
    print(f"per wave (mean): total {tot:.0f} cycles = loop {loop:.0f} + piece prologues {pro:.0f} + "
          f"epilogues/merge/other {tot - loop - pro:.0f}; tiles {st[..., 7].mean():.1f}")
    for grp, sl in (("waves 0-3", slice(0, 4)), ("waves 4-7", slice(4, 8))):
        per = (st[:, sl, :4] / tiles[:, sl, None]).mean(dim=(0, 1))
        print(grp, "cycles/tile:", ", ".join(f"{n} {v:.0f}" for n, v in zip(names, per.tolist())),
              f"| total {per.sum():.0f}", flush=True)
    sys.exit(0)
if len(sys.argv) > 1 and sys.argv[1] == "pmc":
    for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 5):
        run()
    torch.cuda.synchronize()
    sys.exit(0)
fl = 4 * S * S * D
VARIANTS = os.environ.get("ABL", "0,64,1,2,4,8,16,20").split(",")


def timed(dbg, reps=20):
    os.environ["RF_ATTN_DBG"] = dbg
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for _ in range(30):  # clocks settle
    timed("0", 5)
res = {v: [] for v in VARIANTS}
for rnd in range(3):  # interleaved rounds, median (guide rule 24)
    for v in VARIANTS:
        res[v].append(timed(v))
for v in VARIANTS:
    ms = sorted(res[v])[1]
    print(f"dbg={v:>3}: {ms*1e3:7.1f} us  {fl/ms/1e9:7.1f} TF(equiv)  (min {min(res[v])*1e3:.1f})", flush=True)
