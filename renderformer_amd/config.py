"""Model hyper-parameters — same field names/defaults as the reference
``RenderFormerConfig`` (renderformer/models/config.py:5-92) so that an HF
``config.json`` written for the reference loads unchanged.

Defaults are RenderFormer-V1-Base.  ``LARGE_PROXY`` is the assumed
V1.1-swin-large shape (483.9M params, the released config.json is
not available offline).
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import List, Optional


@dataclass(frozen=True)
class RenderFormerConfig:
    # stage 1 (view-independent triangle transformer)
    latent_dim: int = 768
    num_layers: int = 12
    num_heads: int = 6
    dim_feedforward: int = 3072
    num_register_tokens: int = 16
    dropout: float = 0.0
    activation: str = "swiglu"
    norm_type: str = "rms_norm"
    norm_first: bool = True
    view_indep_qk_norm: bool = True
    qk_norm: bool = True
    bias: bool = False
    pe_type: str = "rope"
    rope_type: str = "triangle"
    rope_double_max_freq: bool = False
    vertex_pe_num_freqs: int = 12
    # input encoders
    use_vn_encoder: bool = True
    vn_pe_num_freqs: int = 6
    vn_encoder_norm_type: str = "rms_norm"
    texture_encode_patch_size: int = 32
    texture_channels: int = 13
    texture_encoder_norm_type: str = "rms_norm"
    # stage 2 (view transformer)
    view_transformer_latent_dim: int = 768
    view_transformer_ffn_hidden_dim: int = 3072
    view_transformer_n_heads: int = 6
    view_transformer_n_layers: int = 6
    view_transformer_include_self_attn: bool = True
    view_transformer_use_swin_attn: bool = False
    vdir_pe_type: str = "nerf"
    vdir_num_freqs: int = 0
    patch_size: int = 8
    include_alpha: bool = False
    # DPT decode
    use_dpt_decoder: bool = True
    dpt_features: int = 128
    dpt_out_channels: List[int] = field(default_factory=lambda: [96, 192, 384, 768])
    dpt_out_layers: Optional[List[int]] = None
    turn_to_cam_coord: bool = True
    use_ldr: bool = False

    def get(self, key, default=None):
        return getattr(self, key, default)

    # ------------------------------------------------------------------ helpers
    @property
    def head_dim(self) -> int:
        return self.latent_dim // self.num_heads

    @property
    def vt_head_dim(self) -> int:
        return self.view_transformer_latent_dim // self.view_transformer_n_heads

    @property
    def out_layers(self) -> List[int]:
        n = self.view_transformer_n_layers
        return list(self.dpt_out_layers) if self.dpt_out_layers is not None else list(range(n - 4, n))

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    @classmethod
    def from_dict(cls, d: dict) -> "RenderFormerConfig":
        names = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})

    @classmethod
    def from_json(cls, path: str) -> "RenderFormerConfig":
        with open(path) as f:
            d = json.load(f)
        d = d.get("config", d)  # PyTorchModelHubMixin nests the dataclass under "config"
        return cls.from_dict(d)


BASE = RenderFormerConfig()

LARGE_PROXY = RenderFormerConfig(
    latent_dim=1024, num_layers=14, num_heads=8, dim_feedforward=4096,
    view_transformer_latent_dim=1024, view_transformer_ffn_hidden_dim=4096,
    view_transformer_n_heads=8, view_transformer_n_layers=10,
    view_transformer_use_swin_attn=True,
    dpt_features=256, dpt_out_channels=[128, 256, 512, 1024],
)


def named_config(name: str) -> RenderFormerConfig:
    """Resolve a config by name or by a local snapshot directory containing config.json."""
    if os.path.isdir(name) and os.path.exists(os.path.join(name, "config.json")):
        return RenderFormerConfig.from_json(os.path.join(name, "config.json"))
    table = {
        "renderformer-v1-base": BASE, "base": BASE,
        "renderformer-v1.1-swin-large": LARGE_PROXY, "large": LARGE_PROXY, "large-proxy": LARGE_PROXY,
    }
    key = name.split("/")[-1]
    if key not in table:
        raise ValueError(f"unknown model config {name!r}; pass a local snapshot directory with config.json")
    return table[key]
