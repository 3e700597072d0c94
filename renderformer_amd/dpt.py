"""DPT patch decode (renderformer/layers/dpt.py:174-273) on librfhip's bf16x3 NHWC convolutions.

Layout: every activation is NHWC fp32; the four decoder taps are already NHWC
(token-major patch rows), so no permutes are needed.  Weights are re-laid out
once to [cout_pad][kh][kw][cin_pad] and split into bf16 hi/lo planes.

Graph (dpt.py:242-273), with two exact rewrites:
* FeatureFusionBlock's 1x1 ``out_conv`` is linear and the bilinear resize
  preserves constants, so ``out_conv(resize(x)) == resize(out_conv(x))``: the
  1x1 runs at the lower resolution (4x fewer pixels) before the resize.
* The final ``F.interpolate`` to (hp*patch, wp*patch) is the identity (path_1 is
  already 8*hp with patch 8, align_corners=True) and is skipped; output_conv2's
  SiLU + 1x1 + the ELU + 10^x - 1 decode are fused into the last 3x3 conv.
"""
from __future__ import annotations

from typing import Dict, List

import torch

from ._lib import call, ptr, stream

SILU_IN, SILU_OUT, FINAL, LOG_DECODE, NCHW_OUT = 1, 2, 4, 8, 16


def _split(w: torch.Tensor):
    hi = w.to(torch.bfloat16)
    lo = (w - hi.float()).to(torch.bfloat16)
    return hi.contiguous(), lo.contiguous()


class _Conv:
    def __init__(self, w: torch.Tensor, b, device, deconv: bool = False):
        w = w.detach().float().cpu()
        if deconv:  # ConvTranspose2d weight [cin, cout, k, k] -> [(dy, dx, co), ci]
            cin, cout, k, _ = w.shape
            self.k = k
            mat = w.permute(2, 3, 1, 0).reshape(k * k * cout, cin)
            self.kh = self.kw = 1
            self.cout_pad = k * k * cout
        else:
            cout, cin, kh, kw = w.shape
            self.k = 0
            self.kh, self.kw = kh, kw
            bn = 32 if cout <= 32 else 128
            self.cout_pad = -(-cout // bn) * bn
            mat = w.permute(0, 2, 3, 1)  # [cout, kh, kw, cin]
        self.cin, self.cout = cin, cout
        self.cin_pad = -(-cin // 64) * 64
        if deconv:
            full = torch.zeros(self.cout_pad, self.cin_pad)
            full[:, :cin] = mat
        else:
            full = torch.zeros(self.cout_pad, self.kh, self.kw, self.cin_pad)
            full[:cout, :, :, :cin] = mat
        hi, lo = _split(full.reshape(self.cout_pad, -1))
        self.w_hi, self.w_lo = hi.to(device), lo.to(device)
        self.b = None if b is None else b.detach().float().to(device).contiguous()

    def __call__(self, x: torch.Tensor, stride=1, pad=None, flags=0, res1=None, res2=None, out=None,
                 final=None):
        n, h, w, c = x.shape
        if c != self.cin or x.dtype != torch.float32 or not x.is_contiguous():
            raise ValueError(f"conv input must be contiguous fp32 NHWC with {self.cin} channels, got {tuple(x.shape)}")
        if self.k:
            if out is None:
                out = torch.empty(n, h * self.k, w * self.k, self.cout, device=x.device)
            call("rf_deconv2d_bf16x3", ptr(x), n, h, w, c, ptr(self.w_hi), ptr(self.w_lo), self.cin_pad, self.cout,
                 self.k, ptr(self.b), ptr(out), stream())
            return out
        pad = self.kh // 2 if pad is None else pad
        ho = (h + 2 * pad - self.kh) // stride + 1
        wo = (w + 2 * pad - self.kw) // stride + 1
        w_fin = b_fin = None
        n_fin, alpha = 0, 0.0
        if final is not None:
            w_fin, b_fin, alpha = final
            n_fin = w_fin.shape[0]
        if out is None:
            out = torch.empty(n, ho, wo, n_fin if final is not None else self.cout, device=x.device)
        for r in (res1, res2):
            if r is not None and (r.shape != out.shape or not r.is_contiguous()):
                raise ValueError("residual must match the conv output")
        call("rf_conv2d_bf16x3", ptr(x), n, h, w, c, ptr(self.w_hi), ptr(self.w_lo), self.cin_pad, self.cout,
             self.cout_pad, self.kh, self.kw, stride, pad, ptr(self.b), ptr(res1), ptr(res2), ptr(out), flags,
             ptr(w_fin), ptr(b_fin), n_fin, alpha, stream())
        return out


def upsample(x: torch.Tensor, ho: int, wo: int) -> torch.Tensor:
    n, h, w, c = x.shape
    if (h, w) == (ho, wo):
        return x  # align_corners=True resize to the same size is the identity
    out = torch.empty(n, ho, wo, c, device=x.device)
    call("rf_upsample_bilinear", ptr(x), n, h, w, c, ptr(out), ho, wo, stream())
    return out


class DPTHead:
    def __init__(self, sd: Dict[str, torch.Tensor], prefix: str, device):
        g = lambda n: sd.get(f"{prefix}.{n}")  # noqa: E731
        self.projects = [_Conv(g(f"projects.{i}.weight"), g(f"projects.{i}.bias"), device) for i in range(4)]
        self.resize0 = _Conv(g("resize_layers.0.weight"), g("resize_layers.0.bias"), device, deconv=True)
        self.resize1 = _Conv(g("resize_layers.1.weight"), g("resize_layers.1.bias"), device, deconv=True)
        self.resize3 = _Conv(g("resize_layers.3.weight"), g("resize_layers.3.bias"), device)
        self.rn = [_Conv(g(f"scratch.layer{i + 1}_rn.weight"), None, device) for i in range(4)]
        self.refine = {}
        for r in (1, 2, 3, 4):
            p = f"scratch.refinenet{r}"
            units = {}
            for u in ((1, 2) if r != 4 else (2,)):
                units[u] = [_Conv(g(f"{p}.resConvUnit{u}.conv{c}.weight"), g(f"{p}.resConvUnit{u}.conv{c}.bias"),
                                  device) for c in (1, 2)]
            self.refine[r] = (units, _Conv(g(f"{p}.out_conv.weight"), g(f"{p}.out_conv.bias"), device))
        self.out1 = _Conv(g("scratch.output_conv1.weight"), g("scratch.output_conv1.bias"), device)
        self.out2 = _Conv(g("scratch.output_conv2.0.weight"), g("scratch.output_conv2.0.bias"), device)
        wf = g("scratch.output_conv2.2.weight")
        self.w_fin = wf.detach().float().reshape(wf.shape[0], -1).to(device).contiguous()
        self.b_fin = g("scratch.output_conv2.2.bias").detach().float().to(device).contiguous()
        if self.out2.cout > 32:
            raise ValueError("output_conv2 must have <= 32 channels for the fused head")

    def _rcu_pair(self, convs, x, extra=None):
        """ResidualConvUnit (dpt.py:76-92): conv2(silu(conv1(silu(x)))) + x (+ extra: fusion-block sum)."""
        t = convs[0](x, flags=SILU_IN)
        return convs[1](t, flags=SILU_IN, res1=x, res2=extra)

    def _fuse(self, r, x0, x1, size):
        """FeatureFusionBlock (dpt.py:133-159) with the 1x1 out_conv moved before the resize."""
        units, out_conv = self.refine[r]
        out = x0 if x1 is None else self._rcu_pair(units[1], x1, extra=x0)
        out = self._rcu_pair(units[2], out)
        out = out_conv(out)
        return upsample(out, *size)

    @torch.no_grad()
    def __call__(self, taps: List[torch.Tensor], n_img: int, hp: int, wp: int, patch: int, elu_alpha: float,
                 log_decode: bool, channels_last: bool) -> torch.Tensor:
        layers = []
        for i, t in enumerate(taps):
            x = self.projects[i](t.view(n_img, hp, wp, t.shape[-1]))
            if i == 0:
                x = self.resize0(x)
            elif i == 1:
                x = self.resize1(x)
            elif i == 3:
                x = self.resize3(x, stride=2, pad=1)
            layers.append(x)
        rn = [self.rn[i](layers[i]) for i in range(4)]
        size = lambda t: (t.shape[1], t.shape[2])  # noqa: E731
        p4 = self._fuse(4, rn[3], None, size(rn[2]))
        p3 = self._fuse(3, p4, rn[2], size(rn[1]))
        p2 = self._fuse(2, p3, rn[1], size(rn[0]))
        p1 = self._fuse(1, p2, rn[0], (2 * rn[0].shape[1], 2 * rn[0].shape[2]))
        out = self.out1(p1)
        if (out.shape[1], out.shape[2]) != (hp * patch, wp * patch):
            out = upsample(out, hp * patch, wp * patch)
        flags = FINAL | (LOG_DECODE if log_decode else 0) | (0 if channels_last else NCHW_OUT)
        return self.out2(out, flags=flags, final=(self.w_fin, self.b_fin, elu_alpha))
