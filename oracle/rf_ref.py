"""CPU fp32 restatement of the reference RenderFormer inference path.

TEST INFRASTRUCTURE ONLY — this module is the *checker*, never the product.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it.  The product path (``renderformer_amd``) never imports,
calls or falls back to anything under ``oracle/``.

What it restates (all paths relative to the reference checkout):

* ``renderformer/pipelines/rendering_pipeline.py:28-125``  (log-encode, camera
  transform, ray generation, model call, log-decode)
* ``renderformer/models/renderformer.py:103-206``  (sequence construction,
  register-token centre, stage 1, per-view replication)
* ``renderformer/models/view_transformer.py:88-127``  (ray tokens, stage 2, DPT)
* ``renderformer/layers/attention.py:34-688``  (SwiGLU, MHA with full-width
  q/k RMSNorm, Swin window attention + shift mask, pre-norm layers)
* ``renderformer/layers/dpt.py:57-273``  (DPT head)
* ``renderformer/encodings/rope.py:78-206``  (triangle RoPE, HF half split)
* ``renderformer/encodings/nerf_encoding.py:63-84``  (NeRF sin encoding)
* ``renderformer/utils/ray_generator.py:13-50``, ``utils/transform.py:7-27``

The arithmetic primitives (matmul, SDPA, RMSNorm, conv, bilinear) are the
torch CPU kernels the reference itself calls, so on the same inputs and
weights this restatement agrees with the imported reference to ~1e-6
(pinned by ``tests/test_oracle_golden.py`` against the fixtures written by
``tests/golden/make_golden.py``).

Everything is functional: ``sd`` is a state dict keyed by the reference's
parameter names, ``cfg`` a mapping with the reference
``RenderFormerConfig`` field names.
"""
from __future__ import annotations

import math
from typing import Dict, List, Mapping, Optional

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
EPS = 1e-6  # attention.py:16
WINDOW = 8  # attention.py:604 (TransformerDecoder default window_size)
SHIFT = 4   # attention.py:605


def _c(cfg, key):
    return cfg[key] if isinstance(cfg, Mapping) else getattr(cfg, key)


# ----------------------------------------------------------------------------- encodings
def nerf_encode(x: Tensor, num_freqs: int) -> Tensor:
    """nerf_encoding.py:76-84 (include_input=True, min_freq 0, max_freq L-1)."""
    freqs = 2 ** torch.linspace(0.0, num_freqs - 1, num_freqs)
    scaled = (x[..., None] * freqs).reshape(*x.shape[:-1], -1)
    enc = torch.sin(torch.cat([scaled, scaled + torch.pi / 2.0], dim=-1))
    return torch.cat([x, enc], dim=-1)


def rope_cos_sin(pos: Tensor, freqs: Tensor, head_dim: int):
    """rope.py:315-333 (get_triangle_freqs) + rope.py:78-103 (freqs_to_cos_sin).

    pos [B, S, 9] -> cos, sin [B, 1, S, head_dim]; angle index = coord*nf + f,
    zero padded to head_dim/2 and duplicated (HF half-split layout)."""
    theta = (pos[..., None] * freqs).reshape(pos.shape[0], 1, pos.shape[1], -1)
    half = head_dim // 2
    pad = half - theta.shape[-1]
    if pad < 0:
        raise ValueError("rope angles exceed head_dim/2")  # rope.py:91-92 would crash
    theta = torch.cat([theta, theta.new_zeros(*theta.shape[:-1], pad)], dim=-1)
    theta = torch.cat([theta, theta], dim=-1)
    return theta.cos(), theta.sin()


def rope_apply(t: Tensor, cos: Tensor, sin: Tensor) -> Tensor:
    """rope.py:106-149: t*cos + rotate_half_hf(t)*sin, rotate_half_hf = cat(-x2, x1)."""
    h = t.shape[-1] // 2
    rot = torch.cat([-t[..., h:], t[..., :h]], dim=-1)
    return t * cos + rot * sin


def rms(x: Tensor, w: Tensor, eps: Optional[float]) -> Tensor:
    return F.rms_norm(x, (x.shape[-1],), w, eps)


def linear(x: Tensor, sd, name: str) -> Tensor:
    return F.linear(x, sd[name + ".weight"], sd.get(name + ".bias"))


# ----------------------------------------------------------------------------- attention
def _sdpa(q, k, v, mask):
    return F.scaled_dot_product_attention(q, k, v, attn_mask=mask)


def mha(sd, p: str, q_in: Tensor, kv_in: Tensor, nh: int, key_mask, cos=None, sin=None,
        ctx_cos=None, ctx_sin=None, self_attn=True, qk_norm=True) -> Tensor:
    """attention.py:115-202 (MultiHeadAttention.forward, SDPA branch)."""
    bs, lq, d = q_in.shape
    lk = kv_in.shape[1]
    if self_attn:
        q, k, v = linear(q_in, sd, p + ".in_proj").chunk(3, dim=-1)
    else:
        q = linear(q_in, sd, p + ".q_proj")
        k = linear(kv_in, sd, p + ".k_proj")
        v = linear(kv_in, sd, p + ".v_proj")
    if qk_norm:
        q = rms(q, sd[p + ".q_norm.weight"], EPS)
        k = rms(k, sd[p + ".k_norm.weight"], EPS)
    q = q.view(bs, lq, nh, -1).transpose(1, 2)
    k = k.view(bs, lk, nh, -1).transpose(1, 2)
    v = v.view(bs, lk, nh, -1).transpose(1, 2)
    if cos is not None:
        q = rope_apply(q, cos, sin)
        k = rope_apply(k, ctx_cos if ctx_cos is not None else cos, ctx_sin if ctx_cos is not None else sin)
    mask = None
    if key_mask is not None:
        mask = key_mask.view(bs, 1, 1, lk).expand(-1, nh, -1, -1).reshape(bs, nh, 1, lk)
    o = _sdpa(q, k, v, mask).transpose(1, 2).reshape(bs, lq, d)
    return linear(o, sd, p + ".out_proj")


def swin_region_labels(hp: int, wp: int, ws: int, shift: int) -> Tensor:
    """attention.py:253-265: 3x3 region labels on the *shifted* patch grid."""
    def region(n):
        r = torch.zeros(n, dtype=torch.long)
        r[n - ws:] = 1
        r[n - shift:] = 2
        return r
    return region(hp)[:, None] * 3 + region(wp)[None, :]


def swin_mask(hp: int, wp: int, ws: int, shift: int) -> Tensor:
    """attention.py:237-271: [nW, ws*ws, ws*ws] bool, True = attend."""
    lab = swin_region_labels(hp, wp, ws, shift)
    lab = lab.view(hp // ws, ws, wp // ws, ws).permute(0, 2, 1, 3).reshape(-1, ws * ws)
    return lab[:, None, :] == lab[:, :, None]


def swin_attn(sd, p: str, x: Tensor, hp: int, wp: int, nh: int, shift: int, qk_norm=True) -> Tensor:
    """attention.py:316-370 (SwinSelfAttention.forward)."""
    b, n, c = x.shape
    ws = WINDOW
    g = x.view(b, hp, wp, c)
    if shift:
        g = torch.roll(g, shifts=(-shift, -shift), dims=(1, 2))
    win = g.view(b, hp // ws, ws, wp // ws, ws, c).permute(0, 1, 3, 2, 4, 5).reshape(-1, ws * ws, c)
    nw = win.shape[0]
    q, k, v = linear(win, sd, p + ".in_proj").chunk(3, dim=-1)
    if qk_norm:
        q = rms(q, sd[p + ".q_norm.weight"], EPS)
        k = rms(k, sd[p + ".k_norm.weight"], EPS)
    q = q.view(nw, ws * ws, nh, -1).transpose(1, 2)
    k = k.view(nw, ws * ws, nh, -1).transpose(1, 2)
    v = v.view(nw, ws * ws, nh, -1).transpose(1, 2)
    mask = swin_mask(hp, wp, ws, shift).repeat(b, 1, 1)[:, None] if shift else None
    o = _sdpa(q, k, v, mask).transpose(1, 2).reshape(nw, ws * ws, c)
    o = linear(o, sd, p + ".out_proj")
    o = o.view(b, hp // ws, wp // ws, ws, ws, c).permute(0, 1, 3, 2, 4, 5).reshape(b, hp, wp, c)
    if shift:
        o = torch.roll(o, shifts=(shift, shift), dims=(1, 2))
    return o.reshape(b, n, c)


def swiglu(sd, p: str, x: Tensor) -> Tensor:
    """attention.py:56-57."""
    return linear(F.silu(linear(x, sd, p + ".w1")) * linear(x, sd, p + ".w3"), sd, p + ".w2")


def attention_layer(sd, p, x, nh, key_mask=None, ctx=None, cos=None, sin=None, ctx_cos=None,
                    ctx_sin=None, self_kind=None, hp=None, wp=None, shift=0, qk_norm=True):
    """attention.py:484-527 (AttentionLayer.forward, norm_first, eval)."""
    q = rms(x, sd[p + ".query_norm.weight"], EPS)
    if ctx is None:
        x = x + mha(sd, p + ".multihead_attn", q, q, nh, key_mask, cos, sin, qk_norm=qk_norm)
    else:
        kv = rms(ctx, sd[p + ".kv_norm.weight"], EPS)
        x = x + mha(sd, p + ".multihead_attn", q, kv, nh, key_mask, cos, sin, ctx_cos, ctx_sin,
                    self_attn=False, qk_norm=qk_norm)
    if self_kind is not None:
        h = rms(x, sd[p + ".self_attn_norm.weight"], EPS)
        if self_kind == "swin":
            x = x + swin_attn(sd, p + ".self_attn", h, hp, wp, nh, shift, qk_norm)
        else:
            x = x + mha(sd, p + ".self_attn", h, h, nh, None, cos, sin, qk_norm=qk_norm)
    return x + swiglu(sd, p + ".ffn", rms(x, sd[p + ".ffn_norm.weight"], EPS))


# ----------------------------------------------------------------------------- stages
def center_pos(pos: Tensor, mask: Tensor, n_reg: int):
    """renderformer.py:103-124 (process_tri_vpos_list)."""
    w = (mask.float() / (mask.sum(dim=1, keepdim=True) + 1e-5))[..., None]
    c = (w * pos).sum(dim=1).reshape(-1, 3, 3).mean(dim=1, keepdim=True).repeat(1, n_reg, 3)
    pos = torch.cat([c, pos], dim=1)
    mask = torch.cat([torch.ones(mask.shape[0], n_reg, dtype=torch.bool), mask], dim=1)
    return pos, mask


def construct_seq(sd, cfg, tri_pos, tex, mask, vns):
    """renderformer.py:126-169 (pe_type='rope')."""
    b = tri_pos.shape[0]
    vn_emb = rms(linear(nerf_encode(vns, _c(cfg, "vn_pe_num_freqs")), sd, "vn_encoding_proj"),
                 sd["vn_encoder_norm.weight"], None)
    tex_emb = rms(linear(tex.reshape(b, tex.shape[1], -1), sd, "texture_encoder"),
                  sd["texture_encoder_norm.weight"], None)
    tri = sd["tri_token"] + tex_emb + vn_emb
    seq = torch.cat([sd["reg_tokens"].expand(b, -1, -1), tri], dim=1)
    pos, mask = center_pos(tri_pos, mask, _c(cfg, "num_register_tokens"))
    return seq, mask, pos


def encoder(sd, cfg, seq, mask, pos, taps: Optional[dict] = None):
    """attention.py:579-590 (stage 1)."""
    hd = _c(cfg, "latent_dim") // _c(cfg, "num_heads")
    cos, sin = rope_cos_sin(pos, sd["transformer.rope_emb.freqs"], hd)
    for i in range(_c(cfg, "num_layers")):
        seq = attention_layer(sd, f"transformer.layers.{i}", seq, _c(cfg, "num_heads"), mask, cos=cos,
                              sin=sin, qk_norm=_c(cfg, "view_indep_qk_norm"))
        if taps is not None:
            taps[f"enc{i}"] = seq
    return seq


def dpt_head(sd, p, feats: List[Tensor], hp: int, wp: int, patch: int) -> Tensor:
    """dpt.py:242-273 (+ ResidualConvUnit :76-92, FeatureFusionBlock :133-159)."""
    def conv(x, name, stride=1, pad=None):
        w = sd[name + ".weight"]
        return F.conv2d(x, w, sd.get(name + ".bias"), stride=stride,
                        padding=w.shape[-1] // 2 if pad is None else pad)

    def rcu(x, name):
        o = conv(F.silu(x), name + ".conv1")
        o = conv(F.silu(o), name + ".conv2")
        return o + x

    def fuse(name, x0, x1=None, size=None):
        out = x0
        if x1 is not None:
            out = out + rcu(x1, name + ".resConvUnit1")
        out = rcu(out, name + ".resConvUnit2")
        if size is None:
            out = F.interpolate(out, scale_factor=2, mode="bilinear", align_corners=True)
        else:
            out = F.interpolate(out, size=size, mode="bilinear", align_corners=True)
        return conv(out, name + ".out_conv")

    layers = []
    for i, x in enumerate(feats):
        x = x.permute(0, 2, 1).reshape(x.shape[0], x.shape[-1], hp, wp)
        x = conv(x, f"{p}.projects.{i}")
        if i == 0:
            x = F.conv_transpose2d(x, sd[f"{p}.resize_layers.0.weight"], sd[f"{p}.resize_layers.0.bias"], stride=4)
        elif i == 1:
            x = F.conv_transpose2d(x, sd[f"{p}.resize_layers.1.weight"], sd[f"{p}.resize_layers.1.bias"], stride=2)
        elif i == 3:
            x = conv(x, f"{p}.resize_layers.3", stride=2, pad=1)
        layers.append(x)
    rn = [conv(layers[i], f"{p}.scratch.layer{i + 1}_rn") for i in range(4)]
    s = p + ".scratch"
    path4 = fuse(s + ".refinenet4", rn[3], None, rn[2].shape[2:])
    path3 = fuse(s + ".refinenet3", path4, rn[2], rn[1].shape[2:])
    path2 = fuse(s + ".refinenet2", path3, rn[1], rn[0].shape[2:])
    path1 = fuse(s + ".refinenet1", path2, rn[0], None)
    out = conv(path1, s + ".output_conv1")
    out = F.interpolate(out, (hp * patch, wp * patch), mode="bilinear", align_corners=True)
    out = F.silu(conv(out, s + ".output_conv2.0"))
    return conv(out, s + ".output_conv2.2")


def view_transformer(sd, cfg, cam_o, rays_d, tri_tokens, tri_pos, mask, taps: Optional[dict] = None):
    """view_transformer.py:88-127 (use_dpt_decoder=True, vdir nerf)."""
    pt = _c(cfg, "patch_size")
    bv, hh, ww, _ = rays_d.shape
    hp, wp = hh // pt, ww // pt
    rm = nerf_encode(rays_d, _c(cfg, "vdir_num_freqs")) if _c(cfg, "vdir_num_freqs") > 0 else rays_d
    c = rm.shape[-1]
    tok = rm.view(bv, hp, pt, wp, pt, c).permute(0, 1, 3, 5, 2, 4).reshape(bv, hp * wp, c * pt * pt)
    vt = "view_transformer"
    x = sd[vt + ".ray_map_patch_token"] + rms(linear(tok, sd, vt + ".ray_map_encoder"),
                                             sd[vt + ".ray_map_encoder_norm.weight"], None)
    ray_pos = cam_o[:, None].repeat(1, hp * wp, 3)
    d = _c(cfg, "view_transformer_latent_dim")
    nh = _c(cfg, "view_transformer_n_heads")
    hd = d // nh
    freqs = sd[vt + ".transformer.rope_emb.freqs"]
    cos, sin = rope_cos_sin(ray_pos, freqs, hd)
    ccos, csin = rope_cos_sin(tri_pos, freqs, hd)
    nl = _c(cfg, "view_transformer_n_layers")
    out_layers = _c(cfg, "dpt_out_layers") or list(range(nl - 4, nl))
    swin = _c(cfg, "view_transformer_use_swin_attn")
    self_kind = None if not _c(cfg, "view_transformer_include_self_attn") else ("swin" if swin else "mha")
    feats = []
    for i in range(nl):
        x = attention_layer(sd, f"{vt}.transformer.layers.{i}", x, nh, mask, ctx=tri_tokens, cos=cos, sin=sin,
                            ctx_cos=ccos, ctx_sin=csin, self_kind=self_kind, hp=hp, wp=wp,
                            shift=0 if i % 2 == 0 else SHIFT, qk_norm=_c(cfg, "qk_norm"))
        if taps is not None:
            taps[f"dec{i}"] = x
        if i in out_layers:
            feats.append(x)
    _stamp("stage2_end")
    img = dpt_head(sd, vt + ".out_dpt", feats, hp, wp, pt)
    _stamp("dpt_end")
    if taps is not None:
        taps["dpt"] = img
    return F.elu(img, alpha=1e-3)


def model_forward(sd, cfg, tri_pos, tex, mask, vns, rays_o, rays_d, tri_pos_view, taps=None):
    """renderformer.py:171-206."""
    _stamp("start")
    seq, mask_p, pos = construct_seq(sd, cfg, tri_pos, tex, mask, vns)
    if taps is not None:
        taps["seq0"] = seq
    seq = encoder(sd, cfg, seq, mask_p, pos, taps)
    _stamp("stage1_end")
    b, v = rays_o.shape[:2]
    seq = seq.repeat_interleave(v, dim=0)
    rays_o = rays_o.reshape(-1, *rays_o.shape[2:])
    rays_d = rays_d.reshape(-1, *rays_d.shape[2:])
    tpv = tri_pos_view.reshape(-1, *tri_pos_view.shape[2:])
    m = mask.repeat_interleave(v, dim=0)
    mask_p = mask_p.repeat_interleave(v, dim=0)
    pos_seq, _ = center_pos(tpv, m, _c(cfg, "num_register_tokens"))
    out = view_transformer(sd, cfg, rays_o, rays_d, seq, pos_seq, mask_p, taps)
    return out.view(b, v, *out.shape[1:])


# ----------------------------------------------------------------------------- pipeline
STAMPS: Optional[dict] = None  # bench.py's cpu_baseline sets a dict here to time the stages of one frame


def _stamp(name: str) -> None:
    if STAMPS is not None:
        import time
        STAMPS[name] = time.perf_counter()


def cam_transform(c2w: Tensor, tris: Tensor) -> Tensor:
    """transform.py:7-27 via roma.Rigid: p_cam = R^T p + (-R^T t)."""
    r = c2w[..., :3, :3]
    t = c2w[..., :3, 3]
    rt = r.transpose(-1, -2)
    tinv = -(rt @ t[..., None])[..., 0]
    rt = rt[:, None, None]
    return (rt @ tris[..., None])[..., 0] + tinv[:, None, None]


def ray_gen(c2w: Tensor, fov_rad: Tensor, res: int):
    """ray_generator.py:13-50."""
    bshape = c2w.shape[:-2]
    lin = torch.linspace(0.5, res - 0.5, res, dtype=c2w.dtype)
    x, y = torch.meshgrid(lin, lin, indexing="xy")
    cxy = res / 2
    f = res / 2 / torch.tan(0.5 * fov_rad[..., 0, None, None])
    x = x[None].repeat(*bshape, 1, 1)
    y = y[None].repeat(*bshape, 1, 1)
    dirs = torch.stack([(x - cxy) / f, -(y - cxy) / f, -torch.ones_like(x)], dim=-1)
    r = c2w[..., :3, :3]
    d = torch.sum(dirs[..., None, :] * r[..., None, None, :, :], dim=-1)
    return c2w[..., :3, 3], F.normalize(d, dim=-1, p=2)


@torch.no_grad()
def render(sd, cfg, triangles, texture, mask, vn, c2w, fov, resolution=512, taps=None):
    """rendering_pipeline.py:28-125 on CPU fp32 (autocast is a no-op there).

    Mutates ``texture`` in place exactly like the reference (:67-68)."""
    bs, nv = c2w.shape[:2]
    if _c(cfg, "texture_encode_patch_size") == 1 and texture.dim() == 5:
        texture = texture[:, :, :, 0, 0]
    if not _c(cfg, "use_ldr"):
        texture[:, :, -3:] = torch.log10(texture[:, :, -3:] + 1.0)
    if _c(cfg, "turn_to_cam_coord"):
        tris_v = cam_transform(c2w.reshape(-1, 4, 4), torch.repeat_interleave(triangles, nv, dim=0))
        c2w_v = torch.eye(4, dtype=triangles.dtype).repeat(bs * nv, 1, 1).reshape(bs, nv, 4, 4)
        tris_v = tris_v.reshape(bs, nv, -1, 3, 3)
    else:
        tris_v = triangles.unsqueeze(1).expand(-1, nv, -1, -1, -1)
        c2w_v = c2w
    rays_o, rays_d = ray_gen(c2w_v, fov / 180.0 * torch.pi, resolution)
    if taps is not None:
        taps["rays_d"] = rays_d
        taps["tris_cam"] = tris_v
    out = model_forward(sd, cfg, triangles.reshape(bs, -1, 9), texture, mask, vn.reshape(bs, -1, 9),
                        rays_o, rays_d, tris_v.reshape(bs, nv, -1, 9), taps)
    out = out.permute(0, 1, 3, 4, 2)
    if not _c(cfg, "use_ldr"):
        out = torch.pow(10.0, out) - 1.0
    return out
