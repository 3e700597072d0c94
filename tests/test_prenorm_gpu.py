"""Deferred RMSNorm (rf_prenorm / rf_gemm_add_prenorm / rf_gemm_rownorm, rf.h ABI 15) against fp64 PyTorch
references: the pre-norm of a transformer layer folded into the residual GEMM before it (x * g and the row sums of
squares written from its epilogue) and the projection after it (rows scaled by 1 / rms), on every GEMM loop the
producer / consumer can run (forced tiles: phased 256 / 128x256, phased3 96 / 64 / 128, ring engine 96x256 /
128x128 / 8-wave k64, phased stream-K, ring stream-K), ragged M, and the fallback above 8 column tiles
(reference AttentionLayer.forward pre-norms, renderformer/layers/attention.py:509, 520)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"
EPS = 1e-6


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from renderformer_amd import _lib
    _lib.load()


def _ops():
    from renderformer_amd import ops
    return ops


def relerr(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("m,n", [(1, 256), (333, 768), (5649, 1024), (100, 2048)])
def test_prenorm_row_form(dt, m, n):
    """rf_prenorm: xg = x * g rounded once (bit-equal to torch's RNE cast), slot 0 = sum x^2, slots 1.. = 0."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(m + n)
    x = (torch.randn(m, n, generator=g) * 3).to(dev)
    w = (torch.rand(n, generator=g) + 0.5).to(dev)
    xg = torch.empty(m, n, device=dev, dtype=dt)
    ss = torch.full((m, ops.PRENORM_SLOTS), float("nan"), device=dev)
    ops.prenorm(x, w, xg, ss)
    assert torch.equal(xg, (x * w).to(dt))
    assert relerr(ss[:, 0], (x.double() ** 2).sum(1)) < 1e-6
    assert torch.equal(ss[:, 1:], torch.zeros_like(ss[:, 1:]))


TILES = {"auto": None, "256ph": "256", "128x256ph": "1282", "96x256ph3": "964", "64x256ph3": "645",
         "128x256ph3": "1283", "96x256ring": "962", "128ring8wk64": "12884", "128ring": "128", "skph": "skph",
         "sk512": "sk512"}


def _force(monkeypatch, tile, m, n, k, f16):
    t = TILES[tile]
    if t == "skph":
        monkeypatch.setenv("RF_GEMM_SKPH", "1")
        if n % 256 or k % 64:
            pytest.skip("the phased stream-K loop needs N % 256 == 0 and K % 64 == 0")
    elif t == "sk512":
        if f16:
            pytest.skip("the ring stream-K split is a bf16-operand path")
        monkeypatch.setenv("RF_GEMM_SK", "512")
    elif t:
        if t in ("256", "1282", "964", "645", "1283", "962") and n % 256:
            pytest.skip("256-wide tiles need N % 256 == 0")
        monkeypatch.setenv("RF_GEMM_TILE", t)


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("tile", list(TILES))
@pytest.mark.parametrize("m,n,k", [(1, 256, 64), (777, 512, 192), (5649, 1024, 1024), (4096, 1024, 4096),
                                   (300, 768, 256), (129, 1536, 128)])
def test_gemm_add_prenorm(monkeypatch, dt, tile, m, n, k):
    """Producer: x (fp32) bit-equal to the plain RF_EPI_ADD_F32 GEMM on the same loop, xg = x * g bit-equal to
    torch's cast of the kernel's own x, the slot sums = sum x^2 (N = 1536 > 8 x 128: the GEMM + rf_prenorm)."""
    ops = _ops()
    _force(monkeypatch, tile, m, n, k, dt == torch.float16)
    g = torch.Generator(device="cpu").manual_seed(m + 3 * n + k)
    a = torch.randn(m, k, generator=g).to(dt).to(dev)
    w = (torch.randn(n, k, generator=g) / math.sqrt(k)).to(dt).to(dev)
    x0 = torch.randn(m, n, generator=g).to(dev)
    gw = (torch.rand(n, generator=g) + 0.5).to(dev)
    plain = x0.clone()
    ops.gemm(a, w, plain, None, ops.EPI_ADD_F32)
    x = x0.clone()
    xg = torch.empty(m, n, device=dev, dtype=dt)
    ss = torch.full((m, ops.PRENORM_SLOTS), float("nan"), device=dev)
    ops.gemm_add_prenorm(a, w, x, gw, xg, ss)
    assert torch.equal(x, plain)
    assert relerr(x, x0.double() + a.double() @ w.double().t()) < 1e-5
    assert torch.equal(xg, (x * gw).to(dt))
    assert not torch.isnan(ss).any()
    assert relerr(ss.sum(1), (x.double() ** 2).sum(1)) < 1e-6


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("tile", list(TILES))
@pytest.mark.parametrize("m,n,k", [(1, 256, 256), (777, 512, 512), (5649, 3072, 1024), (4096, 8192, 1024),
                                   (300, 1024, 768)])
def test_gemm_rownorm(monkeypatch, dt, tile, m, n, k):
    """Consumer: rmsnorm(x) @ w.T from (x * g, sum x^2) with the 1 / rms row scale in the epilogue, bf16 / fp16
    outputs and SwiGLU, vs fp64 of the same math (the operands rounded as the kernel rounds them) and vs the
    row-kernel path (rf_rmsnorm + GEMM) within the operands' rounding."""
    ops = _ops()
    _force(monkeypatch, tile, m, n, k, dt == torch.float16)
    from renderformer_amd.model import _interleave_swiglu
    g = torch.Generator(device="cpu").manual_seed(m + 5 * n + k)
    x = (torch.randn(m, k, generator=g) * 4).to(dev)
    gw = (torch.rand(k, generator=g) + 0.5).to(dev)
    w = (torch.randn(n, k, generator=g) / math.sqrt(k)).to(dt).to(dev)
    xg = torch.empty(m, k, device=dev, dtype=dt)
    ss = torch.empty(m, ops.PRENORM_SLOTS, device=dev)
    ops.prenorm(x, gw, xg, ss)
    inv = 1.0 / torch.sqrt((x.double() ** 2).sum(1, keepdim=True) / k + EPS)
    ref = (xg.double() @ w.double().t()) * inv  # the kernel's exact math in fp64
    ref_norm = F.rms_norm(x.double(), (k,), gw.double(), EPS) @ w.double().t()  # the reference's math
    tol16 = 6e-4 if dt == torch.float16 else 4e-3
    for odt in (torch.float16, torch.bfloat16):
        out = torch.empty(m, n, device=dev, dtype=odt)
        ops.gemm_rownorm(xg, w, out, ss, EPS, ops.EPI_BF16)
        otol = 6e-4 if odt == torch.float16 else 4e-3
        assert relerr(out.float(), ref) < otol, odt
        assert relerr(out.float(), ref_norm) < otol + tol16, odt
    h = torch.empty(m, k, device=dev, dtype=dt)
    ops.rmsnorm(x, gw, EPS, h)
    row = torch.empty(m, n, device=dev, dtype=torch.float16)
    ops.gemm(h, w, row, None, ops.EPI_BF16)
    out = torch.empty(m, n, device=dev, dtype=torch.float16)
    ops.gemm_rownorm(xg, w, out, ss, EPS, ops.EPI_BF16)
    assert relerr(out.float(), row.float()) < 2 * tol16
    w13 = _interleave_swiglu(w[: n // 2].cpu(), w[n // 2:].cpu()).to(dev)
    refs = F.silu(ref[:, : n // 2]) * ref[:, n // 2:]
    for odt in (torch.float16, torch.bfloat16):
        outs = torch.empty(m, n // 2, device=dev, dtype=odt)
        ops.gemm_rownorm(xg, w13, outs, ss, EPS, ops.EPI_SWIGLU)
        assert relerr(outs.float(), refs) < (8e-4 if odt == torch.float16 else 5e-3), odt


def test_prenorm_chain_equals_row_kernels():
    """A layer's FFN half through the deferred operands (producer -> consumer, the frame's order) matches the
    row-kernel path (GEMM ADD, rf_rmsnorm, GEMM) on the stage-1 shape."""
    ops = _ops()
    from renderformer_amd.model import _interleave_swiglu
    m, d, f = 5649, 1024, 4096
    g = torch.Generator(device="cpu").manual_seed(11)
    x0 = (torch.randn(m, d, generator=g) * 2).to(dev)
    att = torch.randn(m, d, generator=g).half().to(dev)
    wo = (torch.randn(d, d, generator=g) / math.sqrt(d)).half().to(dev)
    gw = (torch.rand(d, generator=g) + 0.5).to(dev)
    w13 = _interleave_swiglu((torch.randn(f, d, generator=g) / math.sqrt(d)).half(),
                             (torch.randn(f, d, generator=g) / math.sqrt(d)).half()).to(dev)
    x1 = x0.clone()
    ops.gemm(att, wo, x1, None, ops.EPI_ADD_F32)
    h = torch.empty(m, d, device=dev, dtype=torch.float16)
    ops.rmsnorm(x1, gw, EPS, h)
    ref = torch.empty(m, f, device=dev, dtype=torch.float16)
    ops.gemm(h, w13, ref, None, ops.EPI_SWIGLU)
    x2 = x0.clone()
    xg = torch.empty(m, d, device=dev, dtype=torch.float16)
    ss = torch.empty(m, ops.PRENORM_SLOTS, device=dev)
    ops.gemm_add_prenorm(att, wo, x2, gw, xg, ss)
    out = torch.empty(m, f, device=dev, dtype=torch.float16)
    ops.gemm_rownorm(xg, w13, out, ss, EPS, ops.EPI_SWIGLU)
    assert torch.equal(x1, x2)
    assert relerr(out.float(), ref.float()) < 1.5e-3


def test_prenorm_f16_range_flag():
    """An fp16 xg beyond 65504 raises range code 2 (RMSNorm) from the producer epilogue and the row form."""
    ops = _ops()
    m, n, k = 256, 512, 256
    a = torch.randn(m, k, device=dev).half()
    w = (torch.randn(n, k, device=dev) / 16).half()
    gw = torch.ones(n, device=dev)
    xg = torch.empty(m, n, device=dev, dtype=torch.float16)
    ss = torch.empty(m, ops.PRENORM_SLOTS, device=dev)
    for big in (False, True):
        ops.clear_f16_range_flag()
        x = torch.randn(m, n, device=dev)
        if big:
            x[17, 100] = 1e6
        ops.gemm_add_prenorm(a, w, x, gw, xg, ss)
        torch.cuda.synchronize()
        assert ops.f16_range_flag() == (2 if big else 0)
        ops.clear_f16_range_flag()
        ops.prenorm(x, gw, xg, ss)
        torch.cuda.synchronize()
        assert ops.f16_range_flag() == (2 if big else 0)
    ops.clear_f16_range_flag()


@pytest.mark.parametrize("tile", ["auto", "256ph", "96x256ring", "128ring8wk64", "128ring"])
@pytest.mark.parametrize("d", [256, 1024])
def test_gemm_rownorm_segment_sums(monkeypatch, tile, d):
    """seg_ss: per row and segment (q = columns [0, D), k = [D, 2D)) the slot sums equal the sum of squares of
    the values the epilogue wrote (bf16), whatever the column tiling."""
    ops = _ops()
    m, k = 777, 512
    _force(monkeypatch, tile, m, 3 * d, k, True)
    g = torch.Generator(device="cpu").manual_seed(d)
    x = torch.randn(m, k, generator=g).to(dev)
    gw = (torch.rand(k, generator=g) + 0.5).to(dev)
    w = (torch.randn(3 * d, k, generator=g) / math.sqrt(k)).half().to(dev)
    xg = torch.empty(m, k, device=dev, dtype=torch.float16)
    ss = torch.empty(m, ops.PRENORM_SLOTS, device=dev)
    ops.prenorm(x, gw, xg, ss)
    qkv = torch.empty(m, 3 * d, device=dev, dtype=torch.bfloat16)
    seg = torch.full((m, 2, ops.PRENORM_SLOTS), float("nan"), device=dev)
    ops.gemm_rownorm(xg, w, qkv, ss, EPS, seg_ss=seg, seg_w=d)
    plain = torch.empty_like(qkv)
    ops.gemm_rownorm(xg, w, plain, ss, EPS)
    assert torch.equal(qkv, plain)
    assert not torch.isnan(seg).any()
    for s in range(2):
        ref = (qkv[:, s * d:(s + 1) * d].double() ** 2).sum(1)
        assert relerr(seg[:, s].sum(1), ref) < 1e-6


@pytest.mark.parametrize("with_norm", [True])
@pytest.mark.parametrize("shift", [0, 4])
def test_swin_qk_norm_folded(with_norm, shift):
    """rf_swin_attn_fwd_qkn (q/k RMSNorm + q scale on load, from the projection's segment sums) against the unfused
    pair rf_qk_norm_rope + rf_swin_attn_fwd_dt on the same q/k/v: same arithmetic, so equal up to the row sums'
    summation order (a rare last-bit flip of a normalised q/k element)."""
    ops = _ops()
    H, D, n_img, gh, gw_ = 8, 1024, 1, 32, 64
    m, k = n_img * gh * gw_, 256
    g = torch.Generator(device="cpu").manual_seed(7 + shift)
    x = torch.randn(m, k, generator=g).to(dev)
    gx = (torch.rand(k, generator=g) + 0.5).to(dev)
    w = (torch.randn(3 * D, k, generator=g) / math.sqrt(k) * 4).half().to(dev)
    nw = (torch.rand(2 * D, generator=g) + 0.5).to(dev) if with_norm else None
    xg = torch.empty(m, k, device=dev, dtype=torch.float16)
    ss = torch.empty(m, ops.PRENORM_SLOTS, device=dev)
    ops.prenorm(x, gx, xg, ss)
    qkv = torch.empty(m, 3 * D, device=dev, dtype=torch.bfloat16)
    seg = torch.empty(m, 2, ops.PRENORM_SLOTS, device=dev)
    ops.gemm_rownorm(xg, w, qkv, ss, EPS, seg_ss=seg if with_norm else None, seg_w=D)
    ref_qkv = qkv.clone()
    qk = ref_qkv[:, :2 * D]
    ops.qk_norm_rope(qk, qk, H, nw, EPS, n_seg=2, q_scale=ops.Q_LOG2_SCALE)
    out = torch.empty(m, D, device=dev, dtype=torch.float16)
    ref = torch.empty_like(out)
    ops.swin_attention(ref_qkv[:, :D], ref_qkv[:, D:2 * D], ref_qkv[:, 2 * D:], ref, n_img, gh, gw_, shift, H,
                       q_prescaled=True)
    ops.swin_attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], out, n_img, gh, gw_, shift, H,
                       qk_norm=(seg, nw, EPS))
    assert relerr(out.float(), ref.float()) < 1e-3


def test_swin_qk_norm_folded_needs_weights():
    """rf_swin_attn_fwd_qkn refuses a launch without norm weights or row sums (the model takes the unfused pair)."""
    ops = _ops()
    m, D = 4096, 1024
    qkv = torch.zeros(m, 3 * D, device=dev, dtype=torch.bfloat16)
    out = torch.empty(m, D, device=dev, dtype=torch.float16)
    seg = torch.zeros(m, 2, ops.PRENORM_SLOTS, device=dev)
    with pytest.raises(ValueError):
        ops.swin_attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], out, 1, 64, 64, 0, 8, qk_norm=(seg, None, EPS))
