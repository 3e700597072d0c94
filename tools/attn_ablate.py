"""Stage-1 stream-K attention at the bench shape under the RF_ATTN_DBG ablation builds (timing only).

python tools/attn_ablate.py            -> one line per variant
python tools/attn_ablate.py pmc [reps] -> just the shipped kernel, `reps` launches (for rocprofv3 --pmc)
The RF_ATTN_DBG variants (stamps, ablations) exist only in the study build: RF_LIB=renderformer_amd/lib/librfhip_study.so."""
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
# O as fp16 (the frame's instantiation, attn_sk_kernel<true, 0, true, false>: the out-projection's fp16 operand);
# ABL_O=bf16 for the bf16-output kernel
out = torch.empty(S, D, device="cuda", dtype=torch.bfloat16 if os.environ.get("ABL_O") == "bf16" else torch.float16)
prob = torch.tensor([[0, S, 0, S, 0]], dtype=torch.int32, device="cuda")


# cost-balanced stream-K ranges as the model uses them (RF_ATTN_SCHED=0: equal tile counts)
sched = ops.attn_schedule([[0, S, 0, S, 0]], H, out.device)


def run(schedule=sched):
    ops.attention(qs, qkv[:, D:2 * D], qkv[:, 2 * D:], out, prob, S, H, q_prescaled=True, schedule=schedule)


if len(sys.argv) > 1 and sys.argv[1] == "stamps":
    os.environ["RF_ATTN_DBG"] = sys.argv[2] if len(sys.argv) > 2 else "32"
    for _ in range(30):
        run()
    torch.cuda.synchronize()
    ws = ops._attn_workspace(out.device)
    piece = 256 * 128 + 256 * 4  # PIECE_FLOATS (attention.hip): the debug stamps live in the last of 512 slots
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
    # workgroup lifetimes by role in the contiguous stream-K schedule (all workgroups start together, so the
    # spread of lifetimes is the kernel's tail): "mid" = range strictly inside one unit (publishes at its end),
    # "own3" = holds the head of a unit that has a mid piece (merges that late partial), "other"
    nt = (S + 63) // 64
    total = H * ((S + 255) // 256) * nt
    life = st[..., 4].max(dim=1).values  # per workgroup: its slowest wave
    bnd = sched.tolist() if sched is not None else [total * w // 256 for w in range(257)]
    print("schedule:", "cost-balanced" if sched is not None else "equal tiles",
          "tiles per workgroup min/max", min(b - a for a, b in zip(bnd, bnd[1:])), max(b - a for a, b in zip(bnd, bnd[1:])))
    roles = []
    for w in range(256):
        a, b = bnd[w], bnd[w + 1]
        roles.append("empty" if a == b else "mid" if a % nt and a // nt == (b - 1) // nt else "other")
    for w in range(255):
        if roles[w + 1] == "mid" and roles[w] == "other":
            roles[w] = "own3"
    q = torch.tensor([0.5, 0.9, 1.0], dtype=torch.float64)
    print(f"workgroup lifetime (cycles): all p50/p90/max {torch.quantile(life, q).tolist()}")
    for r in ("mid", "own3", "other"):
        sel = torch.tensor([x == r for x in roles])
        if sel.any():
            ep = (st[sel, :, 4] - st[sel, :, :4].sum(-1) - st[sel, :, 6]).mean()
            print(f"  {r:5s} n={int(sel.sum()):3d} lifetime p50/p90/max "
                  f"{[round(v) for v in torch.quantile(life[sel], q).tolist()]}  epilogue/merge mean {ep:.0f}"
                  f"  prologue mean {st[sel, :, 6].mean():.0f}  tiles {st[sel, :, 7].mean():.1f}", flush=True)
    sys.exit(0)
if len(sys.argv) > 1 and sys.argv[1] == "pmc":
    for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 5):
        run()
    torch.cuda.synchronize()
    sys.exit(0)
fl = 4 * S * S * D
VARIANTS = os.environ.get("ABL", "0,u,64,1,2,4,8,16,20").split(",")


def timed(dbg, reps=20):
    """dbg = an RF_ATTN_DBG value, "u": the shipped kernel on equal tile counts (no schedule), "asc": the shipped
    kernel with the round-2 block order (ascending blockIdx inside an XCD group; RF_SK_ASCEND=1, A/B only)"""
    os.environ["RF_ATTN_DBG"] = "0" if dbg in ("u", "asc") else dbg
    os.environ["RF_SK_ASCEND"] = "1" if dbg == "asc" else "0"
    sch = None if dbg == "u" else sched
    run(sch)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run(sch)
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
