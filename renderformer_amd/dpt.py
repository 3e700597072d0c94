"""DPT patch decode (renderformer/layers/dpt.py:174-273) on the device, fp32.

Interim implementation: the convolutions run through PyTorch-ROCm (MIOpen)
in fp32 on the GPU while the HIP implicit-GEMM convolution
is built.  fp32 is mandatory here: the survey measured 2.0e-3 relative L2 for
a bf16 DPT alone, over the 1e-3 parity budget.  The head reads the four
decoder taps straight from the token-major stage-2 buffers (no copies beyond
the NCHW view the convolutions need).
"""
from __future__ import annotations

from typing import Dict, List

import torch
import torch.nn.functional as F


def dpt_weights(sd: Dict[str, torch.Tensor], prefix: str, device) -> Dict[str, torch.Tensor]:
    return {k[len(prefix) + 1:]: v.to(device=device, dtype=torch.float32).contiguous()
            for k, v in sd.items() if k.startswith(prefix + ".")}


def _conv(w, x, name, stride=1, pad=None):
    wt = w[name + ".weight"]
    return F.conv2d(x, wt, w.get(name + ".bias"), stride=stride, padding=wt.shape[-1] // 2 if pad is None else pad)


def _rcu(w, x, name):
    o = _conv(w, F.silu(x), name + ".conv1")
    o = _conv(w, F.silu(o), name + ".conv2")
    return o + x


def _fuse(w, name, x0, x1=None, size=None):
    out = x0
    if x1 is not None:
        out = out + _rcu(w, x1, name + ".resConvUnit1")
    out = _rcu(w, out, name + ".resConvUnit2")
    if size is None:
        out = F.interpolate(out, scale_factor=2, mode="bilinear", align_corners=True)
    else:
        out = F.interpolate(out, size=size, mode="bilinear", align_corners=True)
    return _conv(w, out, name + ".out_conv")


@torch.no_grad()
def dpt_forward(w: Dict[str, torch.Tensor], taps: List[torch.Tensor], n_img: int, hp: int, wp: int,
                patch: int) -> torch.Tensor:
    """taps: 4 x [n_img*hp*wp, D] fp32 token-major -> logits [n_img, out_dim, hp*patch, wp*patch]."""
    layers = []
    for i, t in enumerate(taps):
        x = t.view(n_img, hp, wp, t.shape[-1]).permute(0, 3, 1, 2)
        x = _conv(w, x, f"projects.{i}")
        if i == 0:
            x = F.conv_transpose2d(x, w["resize_layers.0.weight"], w["resize_layers.0.bias"], stride=4)
        elif i == 1:
            x = F.conv_transpose2d(x, w["resize_layers.1.weight"], w["resize_layers.1.bias"], stride=2)
        elif i == 3:
            x = _conv(w, x, "resize_layers.3", stride=2, pad=1)
        layers.append(x)
    rn = [_conv(w, layers[i], f"scratch.layer{i + 1}_rn") for i in range(4)]
    p4 = _fuse(w, "scratch.refinenet4", rn[3], None, rn[2].shape[2:])
    p3 = _fuse(w, "scratch.refinenet3", p4, rn[2], rn[1].shape[2:])
    p2 = _fuse(w, "scratch.refinenet2", p3, rn[1], rn[0].shape[2:])
    p1 = _fuse(w, "scratch.refinenet1", p2, rn[0], None)
    out = _conv(w, p1, "scratch.output_conv1")
    out = F.interpolate(out, (hp * patch, wp * patch), mode="bilinear", align_corners=True)
    out = F.silu(_conv(w, out, "scratch.output_conv2.0"))
    return _conv(w, out, "scratch.output_conv2.2").contiguous()
