"""Algorithmic FLOP counts per rendered frame (2 FLOP per MAC; attention counts QK^T and
PV over valid tokens only).  Used by bench.py for roofline fractions."""
from __future__ import annotations

from .config import RenderFormerConfig


def stage1_layer_flops(cfg: RenderFormerConfig, s: int) -> dict:
    d, f = cfg.latent_dim, cfg.dim_feedforward
    return {"qkv": 2 * s * d * 3 * d, "attn": 4 * s * s * d, "out": 2 * s * d * d, "ffn": 6 * s * d * f}


def stage2_layer_flops(cfg: RenderFormerConfig, s: int, r: int, views: int = 1) -> dict:
    d, f, dc = cfg.view_transformer_latent_dim, cfg.view_transformer_ffn_hidden_dim, cfg.latent_dim
    w = 64 if cfg.view_transformer_use_swin_attn else r
    per_view = {"q": 2 * r * d * d, "cross": 4 * r * s * d, "o": 2 * r * d * d, "ffn": 6 * r * d * f}
    if cfg.view_transformer_include_self_attn:
        per_view.update({"self_qkv": 6 * r * d * d, "self_attn": 4 * r * w * d, "self_out": 2 * r * d * d})
    out = {k: v * views for k, v in per_view.items()}
    out["kv"] = 2 * s * dc * 2 * d  # once per scene (view-independent before RoPE)
    return out


def dpt_flops(cfg: RenderFormerConfig, res: int) -> int:
    p = cfg.patch_size
    hp = res // p
    r = hp * hp
    d, ft, c = cfg.view_transformer_latent_dim, cfg.dpt_features, list(cfg.dpt_out_channels)
    px = [16 * r, 4 * r, r, r // 4]  # pyramid level pixel counts
    tot = sum(2 * r * d * ci for ci in c)
    tot += 2 * px[0] * c[0] * c[0] + 2 * px[1] * c[1] * c[1] + 2 * px[3] * c[3] * c[3] * 9
    tot += sum(2 * px[i] * c[i] * ft * 9 for i in range(4))
    conv = lambda n, pix: n * 2 * pix * ft * ft * 9  # noqa: E731
    tot += conv(2, px[3]) + 2 * px[2] * ft * ft       # refinenet4 (RCU2 only) + out_conv at next size
    tot += conv(4, px[2]) + 2 * px[1] * ft * ft
    tot += conv(4, px[1]) + 2 * px[0] * ft * ft
    tot += conv(4, px[0]) + 2 * (4 * px[0]) * ft * ft
    tot += 2 * res * res * ft * (ft // 2) * 9 + 2 * res * res * (ft // 2) * 32 * 9 + 2 * res * res * 32 * 3
    return tot


def frame_flops(cfg: RenderFormerConfig, n_tris: int, res: int, views: int = 1) -> dict:
    """Per scene with `views` views; divide by views for per-frame numbers."""
    s = n_tris + cfg.num_register_tokens
    r = (res // cfg.patch_size) ** 2
    kt = cfg.texture_channels * cfg.texture_encode_patch_size ** 2
    st1 = stage1_layer_flops(cfg, s)
    st2 = stage2_layer_flops(cfg, s, r, views)
    out = {
        "texture": 2 * n_tris * kt * cfg.latent_dim + 2 * n_tris * 117 * cfg.latent_dim,
        "stage1": cfg.num_layers * sum(st1.values()),
        "stage1_attn": cfg.num_layers * st1["attn"],
        "stage2": cfg.view_transformer_n_layers * sum(st2.values()) + views * 2 * r * 192 * cfg.view_transformer_latent_dim,
        "dpt": views * dpt_flops(cfg, res),
    }
    out["total"] = out["texture"] + out["stage1"] + out["stage2"] + out["dpt"]
    return out
