"""The positional encoding fused into the QK path (rf.h ABI 16): rf_gemm_qk_rope (q/k norm weight +
triangle RoPE in the projection's epilogue, per-row sums of squares), rf_row_rms_scale (the keys' 1 / rms) and
rf_attn_fwd_qn (the queries' 1 / rms as the stream-K attention loads them), each against an fp64 torch restatement of
the reference's q_norm / k_norm + apply_rotary_emb (renderformer/layers/attention.py:127-141, rope.py:106-149), and the
stage-1 stack with and without the fusion against each other and the oracle."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from golden_util import load_case, rel_l2
from oracle import rf_ref

pytestmark = pytest.mark.gpu
dev = "cuda"


def _ops():
    from renderformer_amd import ops
    return ops


def _rope_ref(y, pos, freqs, H):
    """rope_apply of rope_cos_sin on the standard (half-split) layout, fp64; y [M, H*128]."""
    cos, sin = rf_ref.rope_cos_sin(pos.double()[None], freqs.double(), 128)
    return rf_ref.rope_apply(y.view(1, -1, H, 128).transpose(1, 2), cos, sin).transpose(1, 2).reshape(y.shape)


@pytest.mark.parametrize("M,H,norm,f16", [(5649, 8, True, True), (301, 8, True, False), (4096, 8, False, True),
                                          (77, 2, True, True)])
def test_gemm_qk_rope_matches_reference(M, H, norm, f16):
    """out = [rope(g_q * y_q) * q_scale | rope(g_k * y_k) | y_v] in the pair-interleaved column order, y = xg W^T /
    rms (the deferred pre-norm), seg_ss = partial sums of y^2 per q / k row (their total = the full-width sum)."""
    ops = _ops()
    D = H * 128
    K = D
    dt = torch.float16 if f16 else torch.bfloat16
    g = torch.Generator().manual_seed(M + H)
    xg = torch.randn(M, K, generator=g).to(dt)
    w = (torch.randn(3 * D, K, generator=g) / math.sqrt(K)).to(dt)
    ss = (torch.rand(M, ops.PRENORM_SLOTS, generator=g) * K / 4 + 1.0)
    ss[:, 5:] = 0
    gq = torch.rand(2 * D, generator=g) + 0.5
    pos = torch.rand(M, 9, generator=g) * 2 - 1
    freqs = 2 ** torch.linspace(0, math.log2(5), 6)
    perm = ops.rope_pair_perm(D)
    qkp = torch.cat([perm, perm + D, torch.arange(2 * D, 3 * D)])
    out = torch.empty(M, 3 * D, dtype=torch.bfloat16, device=dev)
    seg = torch.zeros(M, 2, ops.PRENORM_SLOTS, device=dev)
    qs = 0.37
    ops.gemm_qk_rope(xg.to(dev), w[qkp].contiguous().to(dev), out, ss.to(dev), 1e-6, D, 2,
                     gq[qkp[:2 * D]].to(dev) if norm else None, seg, pos.to(dev), freqs.to(dev), q_scale=qs)
    # fp64 reference on the standard layout, then the same column permutation
    y = (xg.double() @ w.double().t()) / torch.sqrt(ss.double().sum(1, keepdim=True) / K + 1e-6)
    yq, yk, yv = y[:, :D], y[:, D:2 * D], y[:, 2 * D:]
    zq = _rope_ref(yq * (gq[:D].double() if norm else 1.0), pos, freqs, H) * qs
    zk = _rope_ref(yk * (gq[D:].double() if norm else 1.0), pos, freqs, H)
    ref = torch.cat([zq[:, perm], zk[:, perm], yv], 1)
    got = out.double().cpu()
    for name, a, b in (("q", got[:, :D], ref[:, :D]), ("k", got[:, D:2 * D], ref[:, D:2 * D]),
                       ("v", got[:, 2 * D:], ref[:, 2 * D:])):
        e = float((a - b).norm() / b.norm())
        print(f"{name}: rel L2 {e:.2e}")
        assert e < 5e-3, name  # bf16 output rounding (2^-9) on fp16 / bf16 operands
    if norm:
        sums = seg.sum(-1).double().cpu()
        for s_i, yy in ((0, yq), (1, yk)):
            exp = (yy ** 2).sum(1)
            assert torch.allclose(sums[:, s_i], exp, rtol=2e-3), s_i


def test_row_rms_scale_and_attention_q_scale_match_the_row_kernel_norm():
    """The split norm equals rf_qk_norm_rope's: k rows scaled by 1 / rms from their sums (rf_row_rms_scale) and q rows
    by Q_LOG2_SCALE / rms inside the attention (rf_attn_fwd_qn) give the attention output of q/k normalised up front
    (fp64 reference, softmax scale 1/sqrt(128))."""
    ops = _ops()
    S, H = 1500, 8
    D = H * 128
    g = torch.Generator().manual_seed(3)
    q = torch.randn(S, D, generator=g) * 3
    k = torch.randn(S, D, generator=g) * 2
    v = torch.randn(S, D, generator=g)
    eps = 1e-6
    qss = torch.zeros(S, 2, ops.PRENORM_SLOTS)
    qss[:, 0, :4] = (q.double() ** 2).view(S, 4, -1).sum(-1).float()  # 4 partial sums, slots 4..7 zero
    qss[:, 1, :4] = (k.double() ** 2).view(S, 4, -1).sum(-1).float()
    qkv = torch.cat([q, k, v], 1).bfloat16().to(dev)
    qssd = qss.to(dev)
    ops.row_rms_scale(qkv[:, D:2 * D], qssd[:, 1], eps)
    kk = qkv[:, D:2 * D].double().cpu()
    kref = k.bfloat16().double() / torch.sqrt((k.double() ** 2).mean(1, keepdim=True) + eps)
    assert float((kk - kref).norm() / kref.norm()) < 5e-3
    out = torch.empty(S, D, dtype=torch.bfloat16, device=dev)
    prob = torch.tensor([[0, S, 0, S, 0]], dtype=torch.int32, device=dev)
    sched = ops.attn_schedule([[0, S, 0, S, 0]], H, out.device)
    ops.attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], out, prob, S, H, schedule=sched, q_ss=qssd[:, 0],
                  q_eps=eps)
    qn = q.bfloat16().double() / torch.sqrt((q.double() ** 2).mean(1, keepdim=True) + eps)
    qh, kh, vh = (t.view(S, H, 128).transpose(0, 1) for t in (qn, kk, v.bfloat16().double()))
    ref = (torch.softmax(qh @ kh.transpose(1, 2) / math.sqrt(128), -1) @ vh).transpose(0, 1).reshape(S, D)
    e = float((out.double().cpu() - ref).norm() / ref.norm())
    print(f"attention with the q row scale: rel L2 {e:.2e}")
    assert e < 1e-2


def test_attention_q_ss_equals_prescaled_q():
    """rf_attn_fwd_qn on q with its row factor f applied in-kernel equals rf_attn_fwd_dt on bf16(q * f) bit for bit
    when the factor is exact (a power of two per row: the in-kernel product rounds nothing), across cut units (forced
    small grid)."""
    ops = _ops()
    S, H = 2000, 4
    D = H * 128
    g = torch.Generator().manual_seed(5)
    q = torch.randn(S, D, generator=g).bfloat16().to(dev)
    k = torch.randn(S, D, generator=g).bfloat16().to(dev)
    v = torch.randn(S, D, generator=g).bfloat16().to(dev)
    e2 = torch.randint(-3, 4, (S,), generator=g).double()
    # the kernel computes Q_LOG2_SCALE / sqrt(sum / D + eps): pick sums with rms = 2^-e2 * Q_LOG2_SCALE exactly
    f = 2.0 ** e2 * ops.Q_LOG2_SCALE
    sums = ((ops.Q_LOG2_SCALE / f) ** 2 * D).float()
    qss = torch.zeros(S, ops.PRENORM_SLOTS)
    qss[:, 0] = sums
    qss = qss.to(dev)
    prob = torch.tensor([[0, S, 0, S, 0]], dtype=torch.int32, device=dev)
    o1 = torch.empty(S, D, dtype=torch.bfloat16, device=dev)
    o2 = torch.empty_like(o1)
    ops.attention(q, k, v, o1, prob, S, H, q_ss=qss, q_eps=0.0)
    qp = (q.double() * (2.0 ** e2).to(dev)[:, None]).bfloat16()  # exact: a power of two
    qp = (qp.float() * ops.Q_LOG2_SCALE).bfloat16()
    ops.attention(qp, k, v, o2, prob, S, H, q_prescaled=True)
    err = float((o1.float() - o2.float()).norm() / o2.float().norm())
    print(f"q_ss vs pre-scaled q: rel L2 {err:.2e}")
    assert err < 2e-3


@pytest.mark.parametrize("n_groups,with_norm", [(3, True), (1, False), (10, True)])
def test_qk_norm_rope_groups_ilv_equals_standard_layout(n_groups, with_norm):
    """rf_qk_norm_rope_groups_ilv on rows in the pair-interleaved order (the stage-2 keys when the queries are rotated
    in their projection's epilogue) equals rf_qk_norm_rope_groups on the standard layout, permuted the same way (up to
    the order of the row's sum of squares)."""
    ops = _ops()
    T, H = 211, 8
    D = H * 128
    g = torch.Generator().manual_seed(n_groups)
    kv = torch.randn(T, n_groups * 2 * D, generator=g).bfloat16()
    w = torch.rand(n_groups * D, generator=g) + 0.5
    rows = torch.tensor(list(range(T)) + list(range(0, T, 3)), dtype=torch.int32)
    pos = torch.rand(rows.numel(), 9, generator=g) * 2 - 1
    freqs = 2 ** torch.linspace(0, math.log2(5), 6)
    perm = ops.rope_pair_perm(D)
    cperm = torch.cat([torch.cat([perm + 2 * D * i, torch.arange(D, 2 * D) + 2 * D * i]) for i in range(n_groups)])
    wperm = torch.cat([perm + D * i for i in range(n_groups)])
    std = torch.empty(rows.numel(), n_groups * D, dtype=torch.bfloat16, device=dev)
    ilv = torch.empty_like(std)
    ops.qk_norm_rope_groups(kv.to(dev), 2 * D, std, D, n_groups, H, w.to(dev) if with_norm else None, 1e-6,
                            pos.to(dev), freqs.to(dev), src_rows=rows.to(dev))
    ops.qk_norm_rope_groups(kv[:, cperm].contiguous().to(dev), 2 * D, ilv, D, n_groups, H,
                            w[wperm].to(dev) if with_norm else None, 1e-6, pos.to(dev), freqs.to(dev),
                            src_rows=rows.to(dev), ilv=True)
    a, b = ilv.float().cpu(), std.float().cpu()[:, wperm]
    e = float((a - b).norm() / b.norm())
    print(f"ilv vs standard: rel L2 {e:.2e}, max |diff| {float((a - b).abs().max()):.2e}")
    assert e < 1e-3


def _stage1_rows(fuse, monkeypatch, name="large_cbox_r512"):
    from renderformer_amd import RenderFormer, RenderFormerRenderingPipeline
    monkeypatch.setenv("RF_QK_FUSE", "1" if fuse else "0")
    cfg, sd, inp, res, z = load_case(name)
    pipe = RenderFormerRenderingPipeline(RenderFormer(cfg, sd)).to("cuda")
    assert pipe.model._w.qk_fused == fuse
    d = {k: v.cuda() for k, v in inp.items()}
    out = pipe(d["triangles"], d["texture"].clone(), d["mask"], d["vn"], d["c2w"], d["fov"], resolution=res)
    return out.cpu(), z


def test_qk_fused_matches_unfused_and_reference(monkeypatch):
    """The whole frame at config 2's size with the fused QK path (default: stage 1 and the cross-attention queries) and
    the row-kernel path: both inside the 1e-3 bar of the reference fixture and within 2e-4 of each other (different
    rounding points, same arithmetic)."""
    from golden_util import reference_hdr
    a, z = _stage1_rows(True, monkeypatch)
    b, _ = _stage1_rows(False, monkeypatch)
    hdr, st = reference_hdr(z)
    ea = rel_l2(a[:, :, ::st, ::st], hdr)
    eb = rel_l2(b[:, :, ::st, ::st], hdr)
    d = rel_l2(a, b)
    print(f"fused {ea:.3e}, row kernel {eb:.3e}, fused vs row kernel {d:.3e}")
    assert ea < 1e-3 and eb < 1e-3 and d < 2e-4
