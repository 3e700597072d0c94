"""State-dict schema, deterministic synthetic weights and checkpoint loading.

Parameter names and shapes are those of the reference module tree
(renderformer/models/renderformer.py:13-100,
view_transformer.py:12-86, layers/attention.py:85-482, layers/dpt.py:174-240),
so a reference ``model.safetensors`` loads unchanged and the synthetic state
dict below loads into the reference with ``load_state_dict(strict=True)``.

Synthetic weights are keyed by name: tensor ``name`` is drawn from a CPU
``torch.Generator`` seeded with ``seed * 1_000_003 + crc32(name)``, so any
subset of the model can be regenerated independently and identically on any
host with the same torch build.
"""
from __future__ import annotations

import math
import os
import zlib
from collections import OrderedDict
from typing import Dict, List, Tuple

import torch

from .config import RenderFormerConfig


def rope_freqs(dim: int, double_max_freq: bool = False) -> torch.Tensor:
    """Default triangle-RoPE frequencies (rope.py:171-206 TriangleRotaryEmbedding.__init__)."""
    top = math.log(dim - 1, 2) if double_max_freq else math.log(dim // 2 - 1, 2)
    return 2 ** torch.linspace(0, top, dim // 2)


def _layer_spec(prefix: str, d: int, kv: int, f: int, cross: bool, self_attn: bool, out: List):
    a = prefix + ".multihead_attn"
    if cross:
        out += [(a + ".q_proj.weight", (d, d)), (a + ".k_proj.weight", (d, kv)),
                (a + ".v_proj.weight", (d, kv)), (a + ".out_proj.weight", (d, d))]
    else:
        out += [(a + ".in_proj.weight", (3 * d, d)), (a + ".out_proj.weight", (d, d))]
    out += [(a + ".q_norm.weight", (d,)), (a + ".k_norm.weight", (d,)), (prefix + ".query_norm.weight", (d,))]
    if cross:
        out += [(prefix + ".kv_norm.weight", (kv,))]
    if self_attn:
        s = prefix + ".self_attn"
        out += [(s + ".in_proj.weight", (3 * d, d)), (s + ".out_proj.weight", (d, d)),
                (s + ".q_norm.weight", (d,)), (s + ".k_norm.weight", (d,)),
                (prefix + ".self_attn_norm.weight", (d,))]
    out += [(prefix + ".ffn.w1.weight", (f, d)), (prefix + ".ffn.w2.weight", (d, f)),
            (prefix + ".ffn.w3.weight", (f, d)), (prefix + ".ffn_norm.weight", (d,))]


def param_spec(cfg: RenderFormerConfig) -> "OrderedDict[str, Tuple[int, ...]]":
    """Ordered name -> shape for the supported config family (rope PE, SwiGLU, RMSNorm, no bias, DPT)."""
    if cfg.pe_type != "rope" or cfg.activation != "swiglu" or cfg.norm_type != "rms_norm" or cfg.bias:
        raise ValueError("only pe_type='rope', activation='swiglu', norm_type='rms_norm', bias=False are supported")
    if not cfg.use_dpt_decoder or not cfg.use_vn_encoder:
        raise ValueError("only use_dpt_decoder=True and use_vn_encoder=True are supported")
    d, dv = cfg.latent_dim, cfg.view_transformer_latent_dim
    p = cfg.texture_encode_patch_size
    spec: List = [("tri_token", (1, 1, d)), ("reg_tokens", (1, cfg.num_register_tokens, d))]
    vn_in = 9 * (2 * cfg.vn_pe_num_freqs + 1)
    spec += [("vn_encoding_proj.weight", (d, vn_in)), ("vn_encoding_proj.bias", (d,)), ("vn_encoder_norm.weight", (d,))]
    spec += [("texture_encoder.weight", (d, cfg.texture_channels * p * p)), ("texture_encoder.bias", (d,)),
             ("texture_encoder_norm.weight", (d,))]
    for i in range(cfg.num_layers):
        _layer_spec(f"transformer.layers.{i}", d, d, cfg.dim_feedforward, False, False, spec)
    spec += [("transformer.rope_emb.freqs", (cfg.vertex_pe_num_freqs // 2,))]
    vt = "view_transformer"
    ray_in = 3 * (2 * cfg.vdir_num_freqs + 1) * cfg.patch_size ** 2
    spec += [(vt + ".ray_map_patch_token", (1, 1, dv)), (vt + ".ray_map_encoder.weight", (dv, ray_in)),
             (vt + ".ray_map_encoder.bias", (dv,)), (vt + ".ray_map_encoder_norm.weight", (dv,))]
    for i in range(cfg.view_transformer_n_layers):
        _layer_spec(f"{vt}.transformer.layers.{i}", dv, d, cfg.view_transformer_ffn_hidden_dim, True,
                    cfg.view_transformer_include_self_attn, spec)
    vt_rope = min(cfg.vertex_pe_num_freqs, dv // cfg.view_transformer_n_heads // 18 * 2)  # view_transformer.py:34
    spec += [(vt + ".transformer.rope_emb.freqs", (vt_rope // 2,))]
    # DPT head (dpt.py:174-240)
    o = vt + ".out_dpt"
    ch, ft = list(cfg.dpt_out_channels), cfg.dpt_features
    for i, c in enumerate(ch):
        spec += [(f"{o}.projects.{i}.weight", (c, dv, 1, 1)), (f"{o}.projects.{i}.bias", (c,))]
    spec += [(f"{o}.resize_layers.0.weight", (ch[0], ch[0], 4, 4)), (f"{o}.resize_layers.0.bias", (ch[0],)),
             (f"{o}.resize_layers.1.weight", (ch[1], ch[1], 2, 2)), (f"{o}.resize_layers.1.bias", (ch[1],)),
             (f"{o}.resize_layers.3.weight", (ch[3], ch[3], 3, 3)), (f"{o}.resize_layers.3.bias", (ch[3],))]
    for i, c in enumerate(ch):
        spec += [(f"{o}.scratch.layer{i + 1}_rn.weight", (ft, c, 3, 3))]
    for r in (1, 2, 3, 4):
        rn = f"{o}.scratch.refinenet{r}"
        spec += [(rn + ".out_conv.weight", (ft, ft, 1, 1)), (rn + ".out_conv.bias", (ft,))]
        for u in ((1, 2) if r != 4 else (2,)):
            for cv in (1, 2):
                spec += [(f"{rn}.resConvUnit{u}.conv{cv}.weight", (ft, ft, 3, 3)),
                         (f"{rn}.resConvUnit{u}.conv{cv}.bias", (ft,))]
    spec += [(f"{o}.scratch.output_conv1.weight", (ft // 2, ft, 3, 3)), (f"{o}.scratch.output_conv1.bias", (ft // 2,)),
             (f"{o}.scratch.output_conv2.0.weight", (32, ft // 2, 3, 3)), (f"{o}.scratch.output_conv2.0.bias", (32,)),
             (f"{o}.scratch.output_conv2.2.weight", (3 + int(cfg.include_alpha), 32, 1, 1)),
             (f"{o}.scratch.output_conv2.2.bias", (3 + int(cfg.include_alpha),))]
    return OrderedDict(spec)


def _gen(seed: int, name: str) -> torch.Generator:
    g = torch.Generator(device="cpu")
    g.manual_seed((seed * 1_000_003 + zlib.crc32(name.encode())) % (2 ** 63))
    return g


def synthetic_state_dict(cfg: RenderFormerConfig, seed: int = 0) -> Dict[str, torch.Tensor]:
    """Deterministic random-init weights with the reference's names/shapes (fp32, CPU)."""
    spec = param_spec(cfg)
    sd: Dict[str, torch.Tensor] = OrderedDict()
    for name, shape in spec.items():
        g = _gen(seed, name)
        if name.endswith("rope_emb.freqs"):
            t = rope_freqs(2 * shape[0], cfg.rope_double_max_freq)
        elif name in ("tri_token", "reg_tokens") or name.endswith("ray_map_patch_token"):
            t = torch.randn(shape, generator=g)
        elif "norm" in name.split(".")[-2]:
            t = 1.0 + 0.1 * torch.randn(shape, generator=g)
        elif name.endswith(".bias"):
            w = spec[name[: -len("bias")] + "weight"]
            fan_in = w[0] * math.prod(w[2:]) if "resize_layers.0" in name or "resize_layers.1" in name else math.prod(w[1:])
            b = 1.0 / math.sqrt(fan_in)
            t = (torch.rand(shape, generator=g) * 2 - 1) * b
        else:
            b = 1.0 / math.sqrt(math.prod(shape[1:]))
            t = (torch.rand(shape, generator=g) * 2 - 1) * b
        sd[name] = t.float().contiguous()
    return sd


def load_state_dict_file(path: str) -> Dict[str, torch.Tensor]:
    """Load a reference checkpoint with a loader that executes nothing from the file."""
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path, device="cpu")
    return torch.load(path, map_location="cpu", weights_only=True)


def load_snapshot(path: str) -> Dict[str, torch.Tensor]:
    for fn in ("model.safetensors", "pytorch_model.bin"):
        p = os.path.join(path, fn)
        if os.path.exists(p):
            return load_state_dict_file(p)
    raise FileNotFoundError(f"no model.safetensors / pytorch_model.bin under {path}")


def check_state_dict(cfg: RenderFormerConfig, sd: Dict[str, torch.Tensor], strict: bool = True) -> None:
    spec = param_spec(cfg)
    missing = [k for k in spec if k not in sd]
    bad = [k for k in spec if k in sd and tuple(sd[k].shape) != tuple(spec[k])]
    extra = [k for k in sd if k not in spec]
    if missing or bad or (strict and extra):
        raise ValueError(f"state dict mismatch: missing={missing[:5]} shape={bad[:5]} unexpected={extra[:5]}")
