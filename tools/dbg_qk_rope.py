"""Debug probe of rf_gemm_qk_rope against rf_gemm_rownorm (GPU): the plain, q-scale, norm-weight and RoPE pieces one at
a time, in the pair-interleaved column order.  python tools/dbg_qk_rope.py"""
import math, sys, torch
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from renderformer_amd import ops
dev = "cuda"
M, H = 301, 8
D = H * 128
K = D
g = torch.Generator().manual_seed(1)
xg = torch.randn(M, K, generator=g).half()
w = (torch.randn(3 * D, K, generator=g) / math.sqrt(K)).half()
ss = torch.rand(M, 8, generator=g) * K / 4 + 1.0
pos = torch.rand(M, 9, generator=g) * 2 - 1
freqs = 2 ** torch.linspace(0, math.log2(5), 6)
gq = torch.rand(2 * D, generator=g) + 0.5
base = torch.empty(M, 3 * D, dtype=torch.float16, device=dev)
ops.gemm_rownorm(xg.to(dev), w.to(dev), base, ss.to(dev), 1e-6)
y = base.double().cpu()
def run(norm, p, qs):
    out = torch.empty(M, 3 * D, dtype=torch.bfloat16, device=dev)
    seg = torch.zeros(M, 2, 8, device=dev)
    ops.gemm_qk_rope(xg.to(dev), w.to(dev), out, ss.to(dev), 1e-6, D, 2, gq.to(dev) if norm else None, seg,
                     pos.to(dev) if p else None, freqs.to(dev), q_scale=qs)
    torch.cuda.synchronize()
    return out.double().cpu(), seg.cpu()
def rel(a, b): return float((a - b).norm() / b.norm())
o, _ = run(False, False, 1.0)
print("plain vs rownorm:", rel(o, y), "q", rel(o[:, :D], y[:, :D]), "v", rel(o[:, 2*D:], y[:, 2*D:]))
o, _ = run(False, False, 0.5)
print("q_scale 0.5:", rel(o[:, :D], 0.5 * y[:, :D]), "k", rel(o[:, D:2*D], y[:, D:2*D]))
o, s = run(True, False, 1.0)
print("norm w:", rel(o[:, :2*D], y[:, :2*D] * gq.double()), "sums q", rel(s[:, 0].sum(1).double(), (y[:, :D]**2).sum(1)))
o, _ = run(False, True, 1.0)
# rope in the interleaved layout directly: pairs (2m, 2m+1), angle m
yy = y[:, :2*D].view(M, 2*H, 64, 2)
m = torch.arange(64)
ok = m < 54
pc = torch.where(ok, m // 6, torch.zeros_like(m))
fr = torch.where(ok, freqs.double()[m % 6], torch.zeros(64, dtype=torch.float64))
ang = pos.double()[:, pc] * fr[None, :]   # [M, 64]
c, s_ = ang.cos()[:, None, :], ang.sin()[:, None, :]
x1, x2 = yy[..., 0], yy[..., 1]
r = torch.stack([x1 * c - x2 * s_, x2 * c + x1 * s_], -1).reshape(M, 2 * D)
print("rope:", rel(o[:, :2*D], r), "first row q[:8]", o[0, :8].tolist(), r[0, :8].tolist())
