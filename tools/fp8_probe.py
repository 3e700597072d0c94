"""Probe rf_gemm_mx8's operand / scale layout with structured data (diagnostics)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from renderformer_amd import ops  # noqa: E402
from renderformer_amd.ops import MX8  # noqa: E402

dev = "cuda"


def mk(vals, scales):
    q = vals.to(torch.float8_e4m3fn).view(torch.uint8)
    return MX8(q.contiguous().to(dev), scales.to(torch.uint8).contiguous().to(dev))


def run(name, a, sa, w, sw):
    A, W = mk(a, sa), mk(w, sw)
    out = torch.empty(a.shape[0], w.shape[0], device=dev)
    ops.gemm_mx8(A, W, out, None, ops.EPI_F32)
    ref = (ops.mx8_dequant_ref(A.q.cpu(), A.s.cpu()).double() @ ops.mx8_dequant_ref(W.q.cpu(), W.s.cpu()).double().t())
    o = out.cpu().double()
    err = float((o - ref).norm() / ref.norm())
    print(f"{name}: rel err {err:.3e}", flush=True)
    if err > 1e-5:
        bad = (o - ref).abs() > 1e-3 * ref.abs().max()
        idx = bad.nonzero()[:8].tolist()
        for i, j in idx:
            print(f"   out[{i},{j}] = {o[i, j]:.4f} ref {ref[i, j]:.4f}")
    return out


M = N = 256
K = 128
g = torch.Generator().manual_seed(0)
ones_s = lambda r: torch.full((r, K // 32), 127)  # noqa: E731
a = torch.eye(M, K)
w = (torch.arange(N * K).view(N, K) % 7 - 3).float()
run("A=I(128), W ints, unit scales", a, ones_s(M), w, ones_s(N))
a = torch.randint(-3, 4, (M, K), generator=g).float()
run("A ints, W ints, unit scales", a, ones_s(M), w, ones_s(N))
sa = torch.randint(120, 134, (M, K // 32), generator=g)
run("A ints, W ints, A scales random", a, sa, w, ones_s(N))
sw = torch.randint(120, 134, (N, K // 32), generator=g)
run("A ints, W ints, W scales random", a, ones_s(M), w, sw)
# one K block only non-zero: which block does each lane's scale apply to?
for blk in range(4):
    a2 = torch.zeros(M, K)
    a2[:, blk * 32:(blk + 1) * 32] = 1
    s2 = ones_s(M).clone()
    s2[:, blk] = 128
    run(f"A block {blk} ones (scale x2 on that block)", a2, s2, torch.ones(N, K), ones_s(N))
