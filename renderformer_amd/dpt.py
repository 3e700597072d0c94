"""DPT patch decode (renderformer/layers/dpt.py:174-273) on librfhip's GEMM engine.

Layout: every activation is NHWC.  A tensor that feeds a convolution is kept as
operand planes — optionally of silu(x), the ResidualConvUnit pre-activation —
produced directly by the epilogue of the conv (or resize) that wrote it; tensors
that are also needed as residuals are additionally kept in fp32.

Operand precision (``precision``):
* ``"f16"`` (default): one fp16 plane per operand, one MFMA per product, fp32
  accumulation.  fp16's 11-bit mantissa keeps the DPT at 9e-5 relative L2 on the
  large-proxy config (bf16 operands: 7e-4 there, 2.0e-3 on v1-base — SURVEY
  Appendix C — over the 1e-3 budget).  Activations must stay within fp16 range.
* ``"bf16x3"``: two bf16 planes (hi, lo) per operand and hi*hi + hi*lo + lo*hi,
  fp32-level accuracy at 3x the MFMA work; no range limit beyond fp32's.

Graph with two exact rewrites:
* FeatureFusionBlock's 1x1 ``out_conv`` is linear and the bilinear resize
  preserves constants, so ``out_conv(resize(x)) == resize(out_conv(x))``: the
  1x1 runs at the lower resolution (4x fewer pixels) before the resize.
* The final ``F.interpolate`` to (hp*patch, wp*patch) is the identity (path_1 is
  already 8*hp for patch 8, align_corners=True) and is skipped; output_conv2's
  SiLU + 1x1 + the ELU + 10^x - 1 decode are fused into the last 3x3 conv.
* (fp16 mode) refinenet1's 1x1 ``out_conv`` is folded into ``output_conv1``:
  conv3x3(up(W1 y + b1)) = conv3x3'(up(y)) + a border-class bias, with conv3x3' =
  W3 (x) W1 per tap (``fold_affine_1x1``).  The resize then reads refinenet1's fp16
  planes directly and neither the 1x1 launch nor its fp32 output remain
  (``RF_DPT_FOLD=0`` restores the unfolded path).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

import ctypes

from ._lib import call, ptr, stream

PLANE_SILU, SILU_OUT, FINAL, LOG_DECODE, NCHW_OUT, BORDER_BIAS = 1, 2, 4, 8, 16, 32
BK, BN = 32, 128


def _pad(c: int, m: int) -> int:
    return -(-c // m) * m


def _split(w: torch.Tensor):
    hi = w.to(torch.bfloat16)
    lo = (w - hi.float()).to(torch.bfloat16)
    return hi.contiguous(), lo.contiguous()


@dataclass
class Planes:
    hi: torch.Tensor            # bf16 hi plane, or the one fp16 plane [n, h, w, ld]
    lo: Optional[torch.Tensor]  # bf16 lo plane (None for fp16 planes)
    c: int                      # real channels (ld - c padded channels are zero)

    @property
    def shape(self):
        return self.hi.shape

    @property
    def f16(self) -> bool:
        return self.lo is None

    @staticmethod
    def empty(n, h, w, c, ld, device, f16: bool = False):
        alloc = torch.zeros if ld > c else torch.empty
        if f16:
            return Planes(alloc(n, h, w, ld, dtype=torch.float16, device=device), None, c)
        return Planes(alloc(n, h, w, ld, dtype=torch.bfloat16, device=device),
                      alloc(n, h, w, ld, dtype=torch.bfloat16, device=device), c)


def split_planes(x: torch.Tensor, ld: int, silu: bool = False, f16: bool = False) -> Planes:
    """fp32 NHWC -> operand planes with channel stride ld (bf16 hi/lo, or one fp16 plane)."""
    n, h, w, c = x.shape
    pl = Planes.empty(n, h, w, c, ld, x.device, f16)
    call("rf_split_planes", ptr(x), n * h * w, c, x.stride(2), ptr(pl.hi), ptr(pl.lo), ld, int(silu), stream())
    return pl


def upsample(x: torch.Tensor, ho: int, wo: int, out_f32: bool = True, planes_ld: Optional[int] = None,
             f16: bool = False):
    n, h, w, c = x.shape
    out = torch.empty(n, ho, wo, c, device=x.device) if out_f32 else None
    pl = Planes.empty(n, ho, wo, c, planes_ld, x.device, f16) if planes_ld else None
    call("rf_upsample_bilinear", ptr(x), n, h, w, c, ptr(out), ho, wo, ptr(pl.hi if pl else None),
         ptr(pl.lo if pl else None), planes_ld or 0, stream())
    return out, pl


def upsample_planes(x: Planes, ho: int, wo: int, planes_ld: int) -> Planes:
    """fp16 planes -> bilinear (align_corners=True) fp16 planes of ho x wo (rf_upsample_bilinear_h)."""
    n, h, w, ld = x.shape
    c = _pad(x.c, 8)
    pl = Planes.empty(n, ho, wo, x.c, planes_ld, x.hi.device, True)
    call("rf_upsample_bilinear_h", ptr(x.hi), ld, n, h, w, c, ho, wo, ptr(pl.hi), planes_ld, stream())
    return pl


def conv1x1_group(convs: List["_Conv"], xs: List[Planes], planes_ld: List[int]) -> List[Planes]:
    """Independent fp16 1x1 convolutions over images of one size as ONE launch (rf_conv1x1_f16_group): the
    DPT's four tap projections.  Same results as calling each conv with ``planes_ld``."""
    n, h, w, _ = xs[0].shape
    for c, x in zip(convs, xs):
        if not (c.f16 and x.f16 and c.kh == c.kw == 1 and not c.k and x.shape[:3] == (n, h, w) and
                x.shape[3] == c.cin_pad and x.c == c.cin):
            raise ValueError("conv1x1_group: fp16 1x1 convolutions over equally sized input planes of cin_pad")
    outs = [Planes.empty(n, h, w, c.cout, ld, xs[0].hi.device, True) for c, ld in zip(convs, planes_ld)]
    k = len(convs)

    def arr(ct, vals):
        a = (ct * k)(*vals)
        return ctypes.cast(a, ctypes.c_void_p), a  # (pointer, keep-alive)

    args = [arr(ctypes.c_void_p, [ptr(x.hi) for x in xs]), arr(ctypes.c_int, [c.cin_pad for c in convs]),
            arr(ctypes.c_void_p, [ptr(c.w_hi) for c in convs]), arr(ctypes.c_int, [c.cout for c in convs]),
            arr(ctypes.c_int, [c.cout_pad for c in convs]), arr(ctypes.c_void_p, [ptr(c.b) for c in convs]),
            arr(ctypes.c_void_p, [ptr(o.hi) for o in outs]), arr(ctypes.c_int, list(planes_ld))]
    call("rf_conv1x1_f16_group", k, *[a[0] for a in args], n, h, w, stream())
    return outs


class _ConvDesc(ctypes.Structure):
    """rf.h rf_conv_desc"""
    _fields_ = [(n, ctypes.c_void_p) for n in ("in_", "w", "bias", "out", "p_out")] + \
               [(n, ctypes.c_int) for n in ("n_img", "hi", "wi", "cin_pad", "cout", "cout_pad", "kh", "kw", "stride",
                                            "pad", "deconv_k", "p_ld", "flags")]


def conv_group(jobs: List[dict]) -> List[tuple]:
    """Independent fp16 convolutions / deconvolutions as ONE launch (rf_conv2d_f16_group).  A job is
    dict(conv=_Conv, x=Planes, stride=1, pad=None, out_f32=False, planes_ld=None, planes_silu=False); the
    result per job is (out f32 or None, planes or None), as _Conv.__call__ returns them."""
    descs = (_ConvDesc * len(jobs))()
    results = []
    for d, j in zip(descs, jobs):
        c, x = j["conv"], j["x"]
        n, h, w, ld = x.shape
        if not (c.f16 and x.f16) or ld != c.cin_pad or x.c != c.cin:
            raise ValueError("conv_group: fp16 convolutions whose input planes have cin channels padded to cin_pad")
        stride = j.get("stride", 1)
        pad = c.kh // 2 if j.get("pad") is None else j["pad"]
        if c.k:
            ho, wo = h * c.k, w * c.k
        else:
            ho, wo = (h + 2 * pad - c.kh) // stride + 1, (w + 2 * pad - c.kw) // stride + 1
        out = torch.empty(n, ho, wo, c.cout, device=x.hi.device) if j.get("out_f32") else None
        ld_out = j.get("planes_ld")
        pl = Planes.empty(n, ho, wo, c.cout, ld_out, x.hi.device, True) if ld_out else None
        d.in_, d.w, d.bias, d.out, d.p_out = ptr(x.hi), ptr(c.w_hi), ptr(c.b), ptr(out), ptr(pl.hi if pl else None)
        d.n_img, d.hi, d.wi, d.cin_pad, d.cout, d.cout_pad = n, h, w, c.cin_pad, c.cout, c.cout_pad
        d.kh, d.kw, d.stride, d.pad, d.deconv_k = c.kh, c.kw, stride, pad, c.k
        d.p_ld = ld_out or 0
        d.flags = PLANE_SILU if j.get("planes_silu") else 0
        results.append((out, pl))
    call("rf_conv2d_f16_group", len(jobs), ctypes.cast(descs, ctypes.c_void_p), stream())
    return results


def fold_affine_1x1(w3: torch.Tensor, b3: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor):
    """conv3x3(W3, b3, pad 1)(up(conv1x1(W1, b1)(y))) == conv3x3(W, pad 1)(up(y)) + B[border class]  (exact):
    the per-pixel affine 1x1 commutes with the bilinear resize (which reproduces constants), so the 3x3 sees
    W3 (x) W1 applied to up(y) plus the constant b1, and zero padding cuts b1 out of the taps that fall outside
    the image -- the bias depends on whether the pixel is on the first / last row and column.
    Returns W [cout, cin1, 3, 3] and B [9, cout] (row 3 ry + rx, rf.h RF_CONV_BORDER_BIAS), float64."""
    w3 = w3.detach().double().cpu()
    w1 = w1.detach().double().cpu().reshape(w1.shape[0], w1.shape[1])
    w = torch.einsum("ocyx,ci->oiyx", w3, w1)
    tap = torch.einsum("ocyx,c->oyx", w3, b1.detach().double().cpu())  # b1 through each tap
    keep = {0: [1, 2], 1: [0, 1, 2], 2: [0, 1]}  # class 0: tap 0 reads row / column -1; class 2: tap 2 reads the end
    b = torch.empty(9, w3.shape[0], dtype=torch.float64)
    b3 = b3.detach().double().cpu()
    for ry in range(3):
        for rx in range(3):
            b[3 * ry + rx] = b3 + tap[:, keep[ry]][:, :, keep[rx]].sum((1, 2))
    return w, b


class _Conv:
    """One nn.Conv2d / nn.ConvTranspose2d(kernel == stride) with weights laid out for the engine
    (bf16 hi/lo planes, or one fp16 plane with ``f16``)."""

    def __init__(self, w: torch.Tensor, b, device, deconv: bool = False, f16: bool = False):
        self.f16 = f16
        w = w.detach().float().cpu()
        if deconv:  # ConvTranspose2d weight [cin, cout, k, k] -> rows (dy, dx, co), cols ci
            cin, cout, k, _ = w.shape
            self.k, self.kh, self.kw = k, 1, 1
            self.cin_pad = _pad(cin, BK)
            mat = torch.zeros(k * k * cout, self.cin_pad)
            mat[:, :cin] = w.permute(2, 3, 1, 0).reshape(k * k * cout, cin)
            self.cout_pad = k * k * cout
        else:
            cout, cin, kh, kw = w.shape
            self.k, self.kh, self.kw = 0, kh, kw
            self.cin_pad = _pad(cin, BK)
            # fp16 banks of <= 64 filters (output_conv2) run on the engine's 256x64 tile
            self.cout_pad = 64 if (f16 and cout <= 64) else _pad(cout, BN)
            mat = torch.zeros(self.cout_pad, kh, kw, self.cin_pad)
            mat[:cout, :, :, :cin] = w.permute(0, 2, 3, 1)
            mat = mat.reshape(self.cout_pad, -1)
        self.cin, self.cout = cin, cout
        if f16:
            self.w_hi, self.w_lo = mat.to(torch.float16).contiguous().to(device), None
        else:
            hi, lo = _split(mat)
            self.w_hi, self.w_lo = hi.to(device), lo.to(device)
        self.b = None if b is None else b.detach().float().to(device).contiguous()

    def __call__(self, x: Planes, stride=1, pad=None, res1=None, res2=None, out_f32=False,
                 planes_ld: Optional[int] = None, planes_silu=False, final=None, final_flags=0,
                 border_bias: Optional[torch.Tensor] = None):
        n, h, w, ld = x.shape
        if ld != self.cin_pad or x.c != self.cin:
            raise ValueError(f"conv input planes must have {self.cin} channels padded to {self.cin_pad}, got "
                             f"{x.c}/{ld}")
        if x.f16 != self.f16:
            raise ValueError("conv input planes and weights must use the same operand precision")
        dev = x.hi.device
        from .ops import _gemm_workspace
        ws = _gemm_workspace(dev)
        if self.k:
            ho, wo = h * self.k, w * self.k
        else:
            pad = self.kh // 2 if pad is None else pad
            ho = (h + 2 * pad - self.kh) // stride + 1
            wo = (w + 2 * pad - self.kw) // stride + 1
        if final is not None:
            w_fin, b_fin, alpha = final
            nf = w_fin.shape[0]
            shape = (n, nf, ho, wo) if final_flags & NCHW_OUT else (n, ho, wo, nf)
            out = torch.empty(shape, device=dev)
            if self.f16:
                call("rf_conv2d_f16", ptr(x.hi), n, h, w, ld, ptr(self.w_hi), self.cout, self.cout_pad, self.kh,
                     self.kw, stride, pad, ptr(self.b), 0, 0, ptr(out), 0, 0, FINAL | final_flags, ptr(w_fin),
                     ptr(b_fin), nf, alpha, ptr(ws), ws.numel(), stream())
            else:
                call("rf_conv2d_bf16x3", ptr(x.hi), ptr(x.lo), n, h, w, ld, ptr(self.w_hi), ptr(self.w_lo), self.cout,
                     self.cout_pad, self.kh, self.kw, stride, pad, ptr(self.b), 0, 0, ptr(out), 0, 0, 0,
                     FINAL | final_flags, ptr(w_fin), ptr(b_fin), nf, alpha, ptr(ws), ws.numel(), stream())
            return out
        out = torch.empty(n, ho, wo, self.cout, device=dev) if out_f32 else None
        pl = Planes.empty(n, ho, wo, self.cout, planes_ld, dev, self.f16) if planes_ld else None
        for r in (res1, res2):
            if r is not None and (tuple(r.shape) != (n, ho, wo, self.cout) or not r.is_contiguous()):
                raise ValueError("residual must match the conv output")
        flags = PLANE_SILU if planes_silu else 0
        bias = self.b
        if border_bias is not None:  # [9, cout] rows by border class (fold_affine_1x1)
            if not (self.f16 and not self.k and self.kh == 3 and stride == 1 and pad == 1):
                raise ValueError("border_bias needs an fp16 3x3 stride-1 pad-1 convolution")
            bias, flags = border_bias, flags | BORDER_BIAS
        if self.f16 and self.k:
            call("rf_deconv2d_f16", ptr(x.hi), n, h, w, ld, ptr(self.w_hi), self.cout, self.k, ptr(self.b), ptr(out),
                 ptr(pl.hi if pl else None), planes_ld or 0, ptr(ws), ws.numel(), stream())
        elif self.f16:
            call("rf_conv2d_f16", ptr(x.hi), n, h, w, ld, ptr(self.w_hi), self.cout, self.cout_pad, self.kh, self.kw,
                 stride, pad, ptr(bias), ptr(res1), ptr(res2), ptr(out), ptr(pl.hi if pl else None), planes_ld or 0,
                 flags, 0, 0, 0, 0.0, ptr(ws), ws.numel(), stream())
        elif self.k:
            call("rf_deconv2d_bf16x3", ptr(x.hi), ptr(x.lo), n, h, w, ld, ptr(self.w_hi), ptr(self.w_lo), self.cout,
                 self.k, ptr(self.b), ptr(out), ptr(pl.hi if pl else None), ptr(pl.lo if pl else None),
                 planes_ld or 0, ptr(ws), ws.numel(), stream())
        else:
            call("rf_conv2d_bf16x3", ptr(x.hi), ptr(x.lo), n, h, w, ld, ptr(self.w_hi), ptr(self.w_lo), self.cout,
                 self.cout_pad, self.kh, self.kw, stride, pad, ptr(self.b), ptr(res1), ptr(res2), ptr(out),
                 ptr(pl.hi if pl else None), ptr(pl.lo if pl else None), planes_ld or 0, flags, 0, 0, 0, 0.0,
                 ptr(ws), ws.numel(), stream())
        return out, pl


PRECISIONS = ("f16", "bf16x3")


class DPTHead:
    def __init__(self, sd: Dict[str, torch.Tensor], prefix: str, device, precision: str = "f16"):
        if precision not in PRECISIONS:
            raise ValueError(f"DPT precision must be one of {PRECISIONS}, got {precision!r}")
        self.precision = precision
        f16 = self.f16 = precision == "f16"
        g = lambda n: sd.get(f"{prefix}.{n}")  # noqa: E731
        C = lambda w, b, **kw: _Conv(w, b, device, f16=f16, **kw)  # noqa: E731
        self.projects = [C(g(f"projects.{i}.weight"), g(f"projects.{i}.bias")) for i in range(4)]
        self.resize = {0: C(g("resize_layers.0.weight"), g("resize_layers.0.bias"), deconv=True),
                       1: C(g("resize_layers.1.weight"), g("resize_layers.1.bias"), deconv=True),
                       3: C(g("resize_layers.3.weight"), g("resize_layers.3.bias"))}
        self.rn = [C(g(f"scratch.layer{i + 1}_rn.weight"), None) for i in range(4)]
        self.refine = {}
        for r in (1, 2, 3, 4):
            p = f"scratch.refinenet{r}"
            units = {}
            for u in ((1, 2) if r != 4 else (2,)):
                units[u] = [C(g(f"{p}.resConvUnit{u}.conv{c}.weight"), g(f"{p}.resConvUnit{u}.conv{c}.bias"))
                            for c in (1, 2)]
            self.refine[r] = (units, C(g(f"{p}.out_conv.weight"), g(f"{p}.out_conv.bias")))
        self.out1 = C(g("scratch.output_conv1.weight"), g("scratch.output_conv1.bias"))
        self.out2 = C(g("scratch.output_conv2.0.weight"), g("scratch.output_conv2.0.bias"))
        wf = g("scratch.output_conv2.2.weight")
        self.w_fin = wf.detach().float().reshape(wf.shape[0], -1).to(device).contiguous()
        self.b_fin = g("scratch.output_conv2.2.bias").detach().float().to(device).contiguous()
        if self.out2.cout > 64:
            raise ValueError("output_conv2 must have <= 64 channels for the fused head")
        self.feat_ld = self.refine[1][0][2][0].cin_pad
        # the tap projections as one grouped launch (fp16 mode; RF_DPT_GROUP=0: one launch each)
        self.group_proj = (f16 and os.environ.get("RF_DPT_GROUP", "1") != "0" and len(self.projects) <= 4 and
                           all(c.kh == 1 and c.kw == 1 and not c.k and c.cout_pad % 128 == 0 for c in self.projects))
        # refinenet1's 1x1 out_conv folded into output_conv1 (fp16 mode; module docstring)
        self.fold = f16 and os.environ.get("RF_DPT_FOLD", "1") != "0"
        if self.fold:
            w, b = fold_affine_1x1(g("scratch.output_conv1.weight"), g("scratch.output_conv1.bias"),
                                   g("scratch.refinenet1.out_conv.weight"), g("scratch.refinenet1.out_conv.bias"))
            self.out1_fold = C(w.float(), None)
            self.out1_fold_bias = b.float().to(device).contiguous()

    def _rcu(self, convs, x32, xs: Planes, extra=None, want_f32=False, next_silu=True, next_ld=None):
        """ResidualConvUnit (dpt.py:76-92): conv2(silu(conv1(silu(x)))) + x (+ extra = fusion-block x0)."""
        _, t = convs[0](xs, planes_ld=convs[1].cin_pad, planes_silu=True)
        return convs[1](t, res1=x32, res2=extra, out_f32=want_f32, planes_ld=next_ld, planes_silu=next_silu)

    def _fuse(self, r, x0, x1, x1s, size, last=False):
        """FeatureFusionBlock (dpt.py:133-159) with the 1x1 out_conv moved before the resize."""
        units, out_conv = self.refine[r]
        if x1 is None:
            out, outs = x0, split_planes(x0, self.feat_ld, silu=True, f16=self.f16)
        else:
            out, outs = self._rcu(units[1], x1, x1s, extra=x0, want_f32=True, next_ld=self.feat_ld)
        _, y = self._rcu(units[2], out, outs, next_silu=False, next_ld=out_conv.cin_pad)
        if last and self.fold:  # out_conv lives in output_conv1's folded weights
            return upsample_planes(y, *size, planes_ld=self.out1_fold.cin_pad)
        y32, _ = out_conv(y, out_f32=True)
        if last:
            return upsample(y32, *size, out_f32=False, planes_ld=self.out1.cin_pad, f16=self.f16)[1]
        return upsample(y32, *size)[0]

    def tap_planes(self, i: int, t: torch.Tensor, n_img: int, hp: int, wp: int) -> Planes:
        """Decoder tap i (fp32 patch rows [n_img*hp*wp, C], view_transformer.py:85) -> the operand planes of
        act_postprocess[i]'s 1x1 projection.  Taken when the decoder produces the tap, so the residual
        stream is never cloned (4 x 33.6 MB of copy traffic per 512^2 frame at D = 1024)."""
        return split_planes(t.view(n_img, hp, wp, t.shape[-1]), self.projects[i].cin_pad, f16=self.f16)

    def empty_tap_planes(self, i: int, n_img: int, hp: int, wp: int, c: int, device) -> Planes:
        """The (unfilled) operand planes tap_planes(i, ...) would return, for a producer that writes them itself
        (rf_decoder_forward's taps)."""
        return Planes.empty(n_img, hp, wp, c, self.projects[i].cin_pad, device, self.f16)

    @torch.no_grad()
    def __call__(self, taps: List, n_img: int, hp: int, wp: int, patch: int, elu_alpha: float,
                 log_decode: bool, channels_last: bool) -> torch.Tensor:
        """taps: the four decoder outputs, as fp32 rows or as their tap_planes()."""
        layers = []
        xs = [t if isinstance(t, Planes) else self.tap_planes(i, t, n_img, hp, wp) for i, t in enumerate(taps)]
        nxt_ld = [(self.resize[i] if i in self.resize else self.rn[i]).cin_pad for i in range(len(xs))]
        if self.group_proj:  # the four projections as one launch (their 64^2 GEMMs are latency-bound)
            xs = conv1x1_group(self.projects[:len(xs)], xs, nxt_ld)
        # (the resize layers and layer2-4_rn as grouped launches measured slower: their 32^2 / 64^2 members have
        # K = 4,608 - 9,216, which the stream-K launches spread over the chip and one data-parallel grid does not;
        # same-box frame 83.6 -> 81.3 frames/s, profiles/r3_dpt_group_ab.txt)
        for i, x in enumerate(xs):
            if not self.group_proj:
                _, x = self.projects[i](x, planes_ld=nxt_ld[i])
            if i in self.resize:
                _, x = self.resize[i](x, stride=2 if i == 3 else 1, pad=1 if i == 3 else None,
                                      planes_ld=self.rn[i].cin_pad)
            layers.append(x)
        rn, rns = [], []
        for i in range(4):
            o, s = self.rn[i](layers[i], out_f32=True, planes_ld=self.feat_ld, planes_silu=True)
            rn.append(o)
            rns.append(s)
        size = lambda t: (t.shape[1], t.shape[2])  # noqa: E731
        # refinenet4: only RCU2 on layer4_rn (its input planes hold silu(rn4))
        units4, oc4 = self.refine[4]
        _, y = self._rcu(units4[2], rn[3], rns[3], next_silu=False, next_ld=oc4.cin_pad)
        y32, _ = oc4(y, out_f32=True)
        p4 = upsample(y32, *size(rn[2]))[0]
        p3 = self._fuse(3, p4, rn[2], rns[2], size(rn[1]))
        p2 = self._fuse(2, p3, rn[1], rns[1], size(rn[0]))
        p1 = self._fuse(1, p2, rn[0], rns[0], (2 * rn[0].shape[1], 2 * rn[0].shape[2]), last=True)
        if (p1.shape[1], p1.shape[2]) != (hp * patch, wp * patch):
            raise ValueError("DPT output size mismatch (patch size must be 8)")
        if self.fold:
            _, o1 = self.out1_fold(p1, planes_ld=self.out2.cin_pad, border_bias=self.out1_fold_bias)
        else:
            _, o1 = self.out1(p1, planes_ld=self.out2.cin_pad)
        flags = (LOG_DECODE if log_decode else 0) | (0 if channels_last else NCHW_OUT)
        return self.out2(o1, final=(self.w_fin, self.b_fin, elu_alpha), final_flags=flags)
