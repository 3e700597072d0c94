"""Tensor-level wrappers over the librfhip C ABI.

PyTorch is only plumbing here (device memory, streams): every op validates
shapes/dtypes like the reference's asserts (raising ValueError) and launches a
HIP kernel on the current stream.  Nothing in this module computes on the CPU
or falls back to eager PyTorch math.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from ._lib import call, load, ptr, stream

EPI_BF16, EPI_F32, EPI_ADD_F32, EPI_SWIGLU = 0, 1, 2, 3
_EPI_F16, _EPI_SWIGLU_F16 = 4, 5  # rf.h: the 16-bit epilogues with an fp16 C (chosen from out.dtype)
DT_BF16, DT_F16 = 0, 1
HALF = (torch.bfloat16, torch.float16)  # 16-bit operand formats of the MFMA path
FLT_EPS = float(torch.finfo(torch.float32).eps)  # nn.RMSNorm(eps=None) on fp32 inputs
CUS = 256  # MI355X compute units


class KernelTimer:
    """Times every launch of one tagged op (bench.py roofline): before the launch the library's kernel timer is
    armed (rf_ktimer_arm), so the kernel is dispatched with a start/stop event pair that its own dispatch packet
    timestamps (hipExtLaunchKernel) on the launch stream — the kernel's duration as rocprofv3's kernel trace
    reports it, with no marker packets around the launch."""

    def __init__(self, tag: str):
        self.tag = tag
        self.n = 0

    def start(self, tag):
        if tag != self.tag:
            return None
        call("rf_ktimer_arm")
        self.n += 1
        return None

    def durations_ms(self):
        import ctypes
        buf = (ctypes.c_float * max(self.n, 1))()
        n = int(load().rf_ktimer_read(buf, self.n))
        self.n = 0
        return [float(buf[i]) for i in range(min(n, len(buf)))]


TIMER: Optional[KernelTimer] = None


def _timer_takes(tag: Optional[str], n: int) -> bool:
    """Whether the armed KernelTimer times launches tagged `tag`; if so it counts the n launches that a stage-level
    entry point arms itself (rf_encoder_desc.timer_attn)."""
    if TIMER is None or tag is None or TIMER.tag != tag:
        return False
    TIMER.n += n
    return True


def _t0(tag):
    return TIMER.start(tag) if TIMER is not None and tag is not None else None


def _check(cond, msg):
    if not cond:
        raise ValueError(msg)


def _dev(t, dtype, name):
    _check(t.is_cuda, f"{name} must be a device tensor")
    _check(t.dtype == dtype, f"{name} must be {dtype}, got {t.dtype}")
    _check(t.stride(-1) == 1, f"{name} must be contiguous in its last dim")


_GEMM_WS = {}


def _gemm_workspace(device) -> torch.Tensor:
    """Stream-K partial tiles + flags: one zero-filled buffer per (device, stream), reused by every GEMM on
    that stream, so renders on concurrent streams never share partials or flags."""
    key = (device.type, device.index, torch.cuda.current_stream(device).cuda_stream)
    ws = _GEMM_WS.get(key)
    if ws is None:
        ws = torch.zeros(int(load().rf_gemm_workspace_bytes()), dtype=torch.uint8, device=device)
        _GEMM_WS[key] = ws
    return ws


def clear_device_error() -> None:
    """Recover from a DeviceError: wait for every queued launch, clear the library's device error word and drop
    the stream-K workspaces of this process (fresh zero-filled ones are made on the next launch), so no partial
    or hand-off flag of the failed launch can reach a later one."""
    if torch.cuda.is_available():
        for i in range(torch.cuda.device_count()):
            with torch.cuda.device(i):
                torch.cuda.synchronize()
    load(require_device=False).rf_clear_device_error()
    _GEMM_WS.clear()
    _ATTN_WS.clear()


def f16_range_flag() -> int:
    """The library's fp16 range flag (rf_f16_range_flag, a host-mapped word: no device sync): non-zero once a
    writer of fp16 operands (GEMM epilogue 1, RMSNorm 2, attention O 4, DPT plane 8) met |x| > 65504 (inf included)
    since the last clear.  Read it after the launches in question have completed."""
    return int(load(require_device=False).rf_f16_range_flag())


def clear_f16_range_flag() -> None:
    load(require_device=False).rf_clear_f16_range_flag()


def gemm(a: torch.Tensor, w: torch.Tensor, out: torch.Tensor, bias: Optional[torch.Tensor] = None,
         epilogue: int = EPI_BF16, tag: Optional[str] = None, flag: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out (epilogue)= a @ w.T ; a [M,K], w [N,K] both bf16 (rf_gemm_bf16) or both fp16 (rf_gemm_f16).  The
    16-bit epilogues (EPI_BF16, EPI_SWIGLU) write out's dtype (bf16 or fp16).  With ``flag`` (int32 device
    scalar; bf16 only) the launch is a no-op unless the flag is non-zero when it runs (rf_gemm_bf16_if)."""
    _check(a.dtype in HALF and w.dtype == a.dtype, f"gemm: a/w must both be bf16 or both fp16 ({a.dtype}, {w.dtype})")
    _dev(a, a.dtype, "a")
    _dev(w, w.dtype, "w")
    m, k = a.shape
    n, k2 = w.shape
    _check(k == k2, f"gemm: K mismatch {k} vs {k2}")
    if epilogue in (EPI_BF16, EPI_SWIGLU):
        _check(out.dtype in HALF, "gemm: 16-bit epilogue needs a bf16 or fp16 out")
        _dev(out, out.dtype, "out")
    else:
        _dev(out, torch.float32, "out")
    ncols = n // 2 if epilogue == EPI_SWIGLU else n
    _check(out.shape[0] == m and out.shape[1] == ncols, f"gemm: out shape {tuple(out.shape)} != ({m}, {ncols})")
    if bias is not None:
        _dev(bias, torch.float32, "bias")
    ws = _gemm_workspace(a.device)
    epi = epilogue
    if out.dtype == torch.float16:
        epi = _EPI_F16 if epilogue == EPI_BF16 else _EPI_SWIGLU_F16
    _t0(tag)
    if flag is None:
        call("rf_gemm_f16" if a.dtype == torch.float16 else "rf_gemm_bf16", ptr(a), a.stride(0), ptr(w), w.stride(0),
             ptr(out), out.stride(0), ptr(bias), m, n, k, epi, ptr(ws), ws.numel(), stream())
    else:
        _check(a.dtype == torch.bfloat16 and out.dtype != torch.float16, "gemm: the gated form is bf16 only")
        _dev(flag, torch.int32, "flag")
        call("rf_gemm_bf16_if", ptr(flag), ptr(a), a.stride(0), ptr(w), w.stride(0), ptr(out), out.stride(0),
             ptr(bias), m, n, k, epilogue, ptr(ws), ws.numel(), stream())
    return out


class MX8:
    """An MX fp8 operand: e4m3 bytes q [rows, K] (uint8) + E8M0 block scales s [rows, K/32] (uint8)."""
    __slots__ = ("q", "s")

    def __init__(self, q: torch.Tensor, s: torch.Tensor):
        self.q, self.s = q, s

    @property
    def shape(self):
        return self.q.shape

    @classmethod
    def empty(cls, rows: int, cols: int, device) -> "MX8":
        return cls(torch.empty(rows, cols, dtype=torch.uint8, device=device),
                   torch.empty(rows, cols // 32, dtype=torch.uint8, device=device))


def quant_mx8(x: torch.Tensor, out: Optional[MX8] = None) -> MX8:
    """bf16 rows -> MX fp8 (rf_quant_mx8: per-32 E8M0 scale 2^ceil(log2(amax/448)), RNE e4m3)."""
    _dev(x, torch.bfloat16, "x")
    rows, cols = x.shape
    out = out or MX8.empty(rows, cols, x.device)
    _check(out.q.shape == (rows, cols) and out.s.shape[0] == rows, "quant_mx8: output shape")
    call("rf_quant_mx8", ptr(x), x.stride(0), rows, cols, ptr(out.q), out.q.stride(0), ptr(out.s), out.s.stride(0),
         stream())
    return out


def gemm_mx8(a: MX8, w: MX8, out: torch.Tensor, bias: Optional[torch.Tensor] = None, epilogue: int = EPI_BF16,
             tag: Optional[str] = None) -> torch.Tensor:
    """out (epilogue)= dequant(a) @ dequant(w).T on the block-scaled fp8 MFMA (rf_gemm_mx8)."""
    for t, n in ((a.q, "a"), (w.q, "w"), (a.s, "a scales"), (w.s, "w scales")):
        _dev(t, torch.uint8, n)
    m, k = a.q.shape
    n, k2 = w.q.shape
    _check(k == k2, f"gemm_mx8: K mismatch {k} vs {k2}")
    want = torch.bfloat16 if epilogue in (EPI_BF16, EPI_SWIGLU) else torch.float32
    _dev(out, want, "out")
    ncols = n // 2 if epilogue == EPI_SWIGLU else n
    _check(out.shape[0] == m and out.shape[1] == ncols, f"gemm_mx8: out shape {tuple(out.shape)} != ({m}, {ncols})")
    if bias is not None:
        _dev(bias, torch.float32, "bias")
    _t0(tag)
    call("rf_gemm_mx8", ptr(a.q), a.q.stride(0), ptr(a.s), a.s.stride(0), ptr(w.q), w.q.stride(0), ptr(w.s),
         w.s.stride(0), ptr(out), out.stride(0), ptr(bias), m, n, k, epilogue, stream())
    return out


def mx8_dequant_ref(q: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    """fp32 value of an MX fp8 tensor (any device; for tests and weight checks)."""
    v = q.view(torch.float8_e4m3fn).float()
    scale = torch.pow(2.0, s.float() - 127.0)
    return (v.view(v.shape[0], -1, 32) * scale[:, :, None]).view(v.shape)


def mx8_quant_ref(x: torch.Tensor):
    """Reference MX quantisation on any device (torch float8_e4m3fn casts, RNE): the same rule as rf_quant_mx8.
    Used for the weights at load time and as the tests' oracle for the device quantiser."""
    rows, cols = x.shape
    xb = x.float().view(rows, cols // 32, 32)
    amax = xb.abs().amax(-1)
    m, ex = torch.frexp(amax)
    e = ex - 9 + (m > 0.875).to(ex.dtype)
    e = torch.where(amax > 0, e, torch.full_like(e, -127)).clamp(-127, 127)
    q = (xb * torch.pow(2.0, -e.float())[:, :, None]).to(torch.float8_e4m3fn).view(rows, cols)
    return q.view(torch.uint8), (e + 127).to(torch.uint8)


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor) -> torch.Tensor:
    """out (bf16 or fp16, the next GEMM's operand format) = RMSNorm(x f32) * w."""
    _dev(x, torch.float32, "x")
    _check(out.dtype in HALF, "rmsnorm: out must be bf16 or fp16")
    _dev(out, out.dtype, "out")
    _check(x.shape == out.shape and w.numel() == x.shape[1], "rmsnorm: shape mismatch")
    call("rf_rmsnorm_f16" if out.dtype == torch.float16 else "rf_rmsnorm", ptr(x), x.stride(0), ptr(w), eps, ptr(out),
         out.stride(0), x.shape[0], x.shape[1], stream())
    return out


PRENORM_SLOTS = 8  # rf.h RF_PRENORM_SLOTS: partial sums of squares per row of a deferred RMSNorm


def _dt(t: torch.Tensor) -> int:
    return 1 if t.dtype == torch.float16 else 0  # RF_DT_F16 / RF_DT_BF16


def prenorm(x: torch.Tensor, w: torch.Tensor, xg: torch.Tensor, ss: torch.Tensor) -> torch.Tensor:
    """Deferred RMSNorm, row form (rf_prenorm): xg = x * w in xg's dtype (bf16 / fp16) and the row sums of x^2 in
    ss [rows, PRENORM_SLOTS] (slot 0); gemm_rownorm(xg, ...) then equals gemm(rmsnorm(x, w), ...)."""
    _dev(x, torch.float32, "x")
    _check(xg.dtype in HALF, "prenorm: xg must be bf16 or fp16")
    _dev(xg, xg.dtype, "xg")
    _dev(ss, torch.float32, "ss")
    _check(xg.shape == x.shape and w.numel() == x.shape[1], "prenorm: shape mismatch")
    _check(ss.shape[0] >= x.shape[0] and ss.shape[1] == PRENORM_SLOTS and ss.is_contiguous(), "prenorm: ss shape")
    call("rf_prenorm", ptr(x), x.stride(0), ptr(w), ptr(xg), xg.stride(0), ptr(ss), x.shape[0], x.shape[1], _dt(xg),
         stream())
    return xg


def gemm_add_prenorm(a: torch.Tensor, w: torch.Tensor, x: torch.Tensor, norm_w: torch.Tensor, xg: torch.Tensor,
                     ss: torch.Tensor, tag: Optional[str] = None) -> torch.Tensor:
    """x += a @ w.T (fp32 residual) and, from the same epilogue, the next pre-norm's operands: xg = x * norm_w and
    the row sums of squares ss (rf_gemm_add_prenorm; a / w / xg all bf16 or all fp16)."""
    _check(a.dtype in HALF and w.dtype == a.dtype and xg.dtype == a.dtype,
           f"gemm_add_prenorm: a / w / xg must share bf16 or fp16 ({a.dtype}, {w.dtype}, {xg.dtype})")
    for t, n in ((a, "a"), (w, "w"), (xg, "xg")):
        _dev(t, t.dtype, n)
    _dev(x, torch.float32, "x")
    _dev(ss, torch.float32, "ss")
    m, k = a.shape
    n, k2 = w.shape
    _check(k == k2 and x.shape == (m, n) and xg.shape == (m, n) and norm_w.numel() == n,
           "gemm_add_prenorm: shape mismatch")
    _check(ss.shape[0] >= m and ss.shape[1] == PRENORM_SLOTS and ss.is_contiguous(), "gemm_add_prenorm: ss shape")
    ws = _gemm_workspace(a.device)
    _t0(tag)
    call("rf_gemm_add_prenorm", ptr(a), a.stride(0), ptr(w), w.stride(0), ptr(x), x.stride(0), m, n, k, ptr(norm_w),
         ptr(xg), xg.stride(0), ptr(ss), _dt(a), ptr(ws), ws.numel(), stream())
    return x


def gemm_rownorm(xg: torch.Tensor, w: torch.Tensor, out: torch.Tensor, ss: torch.Tensor, eps: float,
                 epilogue: int = EPI_BF16, tag: Optional[str] = None, seg_ss: Optional[torch.Tensor] = None,
                 seg_w: int = 0) -> torch.Tensor:
    """out (epilogue)= rmsnorm(x) @ w.T from the deferred form (rf_gemm_rownorm): xg = x * g and ss from prenorm /
    gemm_add_prenorm; the rows are scaled by 1 / rms(x) in the epilogue (EPI_BF16 or EPI_SWIGLU; out bf16 / fp16).
    With ``seg_ss`` [M, n_seg, PRENORM_SLOTS] (EPI_BF16 only) also the partial sums of the squares of the written
    values per segment of ``seg_w`` columns: the row sums of a following full-width q/k RMSNorm (swin_attention's
    ``qk_norm``)."""
    _check(xg.dtype in HALF and w.dtype == xg.dtype, "gemm_rownorm: xg / w must both be bf16 or both fp16")
    _check(epilogue in (EPI_BF16, EPI_SWIGLU), "gemm_rownorm: epilogue must be EPI_BF16 or EPI_SWIGLU")
    _dev(xg, xg.dtype, "xg")
    _dev(w, w.dtype, "w")
    _dev(ss, torch.float32, "ss")
    _check(out.dtype in HALF, "gemm_rownorm: out must be bf16 or fp16")
    _dev(out, out.dtype, "out")
    m, k = xg.shape
    n, k2 = w.shape
    ncols = n // 2 if epilogue == EPI_SWIGLU else n
    _check(k == k2 and out.shape == (m, ncols), "gemm_rownorm: shape mismatch")
    _check(ss.shape[0] >= m and ss.shape[1] == PRENORM_SLOTS and ss.is_contiguous(), "gemm_rownorm: ss shape")
    epi = epilogue
    if out.dtype == torch.float16:
        epi = _EPI_F16 if epilogue == EPI_BF16 else _EPI_SWIGLU_F16
    ws = _gemm_workspace(xg.device)
    _t0(tag)
    n_seg = 0
    if seg_ss is not None:
        _dev(seg_ss, torch.float32, "seg_ss")
        _check(epilogue == EPI_BF16 and seg_ss.is_contiguous() and seg_ss.dim() == 3 and seg_ss.shape[0] >= m
               and seg_ss.shape[2] == PRENORM_SLOTS and seg_w > 0, "gemm_rownorm: seg_ss [M, n_seg, 8] with EPI_BF16")
        n_seg = seg_ss.shape[1]
    call("rf_gemm_rownorm", ptr(xg), xg.stride(0), ptr(w), w.stride(0), ptr(out), out.stride(0), m, n, k, epi, ptr(ss),
         k, eps, ptr(seg_ss), seg_w, n_seg, _dt(xg), ptr(ws), ws.numel(), stream())
    return out


def qk_norm_rope(src: torch.Tensor, dst: torch.Tensor, n_heads: int, norm_w: Optional[torch.Tensor], eps: float,
                 pos: Optional[torch.Tensor] = None, freqs: Optional[torch.Tensor] = None, pos_div: int = 1,
                 src_rows: Optional[torch.Tensor] = None, n_seg: int = 1, q_scale: float = 1.0,
                 ilv: bool = False) -> torch.Tensor:
    """dst[r] = rope(rmsnorm(src[src_rows[r]])) over the full width (attention.py:127-141), for n_seg
    consecutive width-(n_heads*128) segments (q and k of a qkv row) with weights norm_w [n_seg*dim].
    Segment 0 is also multiplied by q_scale (Q_LOG2_SCALE pre-scales q for attention(scale=LN2)).
    ilv: rows (and norm_w) in rope_pair_perm's pair-interleaved order (rf_qk_norm_rope_groups_ilv)."""
    _dev(src, torch.bfloat16, "src")
    _dev(dst, torch.bfloat16, "dst")
    rows, width = dst.shape
    dim = n_heads * 128
    _check(width == n_seg * dim and src.shape[1] == width, "qk_norm_rope: width mismatch")
    if src_rows is None:
        _check(src.shape[0] == rows, "qk_norm_rope: row mismatch")
    else:
        _dev(src_rows, torch.int32, "src_rows")
    if norm_w is not None:
        _check(norm_w.numel() == n_seg * dim, "qk_norm_rope: norm weight size")
    if pos is not None:
        _dev(pos, torch.float32, "pos")
        _check(pos.shape[1] == 9 and freqs is not None, "qk_norm_rope: pos must be [*, 9] with freqs")
    if ilv:  # one group of n_seg segments
        call("rf_qk_norm_rope_groups_ilv", ptr(src), src.stride(0), 0, ptr(dst), dst.stride(0), 0, ptr(src_rows), rows,
             dim, n_heads, n_seg, 1, ptr(norm_w), 0, eps, q_scale, ptr(pos), pos.stride(0) if pos is not None else 0,
             pos_div, ptr(freqs), freqs.numel() if freqs is not None else 0, stream())
        return dst
    call("rf_qk_norm_rope", ptr(src), src.stride(0), ptr(dst), dst.stride(0), ptr(src_rows), rows, dim, n_heads,
         n_seg, ptr(norm_w), eps, q_scale, ptr(pos), pos.stride(0) if pos is not None else 0, pos_div, ptr(freqs),
         freqs.numel() if freqs is not None else 0, stream())
    return dst


def qk_norm_rope_groups(src: torch.Tensor, src_gstride: int, dst: torch.Tensor, dst_gstride: int, n_groups: int,
                        n_heads: int, norm_w: Optional[torch.Tensor], eps: float, pos: Optional[torch.Tensor] = None,
                        freqs: Optional[torch.Tensor] = None, src_rows: Optional[torch.Tensor] = None,
                        seg0_scale: float = 1.0, ilv: bool = False) -> torch.Tensor:
    """qk_norm_rope (one segment) on n_groups column groups in one launch: group g maps the width-
    (n_heads*128) block at column g*src_gstride of src to column g*dst_gstride of dst with norm weights
    norm_w[g*dim:(g+1)*dim].  src/dst are the full row matrices holding every group.  Every group is also
    multiplied by seg0_scale (qk_norm_rope's q_scale, applied per group: rf.h)."""
    _dev(src, torch.bfloat16, "src")
    _dev(dst, torch.bfloat16, "dst")
    dim = n_heads * 128
    rows = dst.shape[0]
    _check(n_groups >= 1 and (n_groups - 1) * src_gstride + dim <= src.shape[1]
           and (n_groups - 1) * dst_gstride + dim <= dst.shape[1], "qk_norm_rope_groups: groups exceed the width")
    if src_rows is None:
        _check(src.shape[0] == rows, "qk_norm_rope_groups: row mismatch")
    else:
        _dev(src_rows, torch.int32, "src_rows")
        _check(src_rows.numel() == rows, "qk_norm_rope_groups: src_rows size")
    if norm_w is not None:
        _check(norm_w.numel() == n_groups * dim, "qk_norm_rope_groups: norm weight size")
    if pos is not None:
        _dev(pos, torch.float32, "pos")
        _check(pos.shape[1] == 9 and freqs is not None, "qk_norm_rope_groups: pos must be [*, 9] with freqs")
    call("rf_qk_norm_rope_groups_ilv" if ilv else "rf_qk_norm_rope_groups", ptr(src), src.stride(0), src_gstride,
         ptr(dst), dst.stride(0), dst_gstride,
         ptr(src_rows), rows, dim, n_heads, 1, n_groups, ptr(norm_w), dim, eps, float(seg0_scale), ptr(pos),
         pos.stride(0) if pos is not None else 0, 1, ptr(freqs), freqs.numel() if freqs is not None else 0, stream())
    return dst


ATTN_QBLK = 128 if os.environ.get("RF_ATTN_KERNEL", "3") == "2" else 256  # query rows per legacy workgroup
LN2 = math.log(2.0)
# softmax scale * log2(e) for head_dim 128: q pre-multiplied by this (qk_norm_rope q_scale) lets attention run
# with scale = ln 2, i.e. scores are exp2 exponents and the kernel needs no per-score multiply
Q_LOG2_SCALE = 1.0 / math.sqrt(128) / LN2
_ATTN_WS = {}


def _attn_workspace(device) -> torch.Tensor:
    """Stream-K partials + per-workgroup flags, zero-filled once per (device, stream) (the kernel re-arms the
    flags; rf.h allows one launch at a time per workspace, so concurrent streams each get their own)."""
    key = (device.type, device.index, torch.cuda.current_stream(device).cuda_stream)
    ws = _ATTN_WS.get(key)
    if ws is None:
        nbytes = load().rf_attn_workspace_bytes(0, 1, 0)
        ws = torch.zeros((nbytes + 3) // 4, dtype=torch.float32, device=device)
        _ATTN_WS[key] = ws
    return ws


def attn_grid(device=None) -> int:
    """Workgroups of the stream-K attention grid: RF_ATTN_GRID (tests) or the device's CU count."""
    env = os.environ.get("RF_ATTN_GRID")
    if env:
        return int(env)
    with torch.cuda.device(device):
        return int(load().rf_attn_grid())


def attn_schedule_host(problems, n_heads: int, grid: int):
    """rf_attn_schedule (host only, no device): cost-balanced stream-K range bounds, int64 numpy [grid + 1]."""
    import numpy as np
    arr = np.ascontiguousarray(np.asarray(problems, dtype=np.int32).reshape(-1, 5))
    out = np.zeros(grid + 1, dtype=np.int64)
    lib = load(require_device=False)
    rc = lib.rf_attn_schedule(arr.ctypes.data, arr.shape[0], n_heads, grid, out.ctypes.data)
    if rc != 0:
        raise ValueError(lib.rf_last_error().decode(errors="replace"))
    return out


def attn_schedule_enabled() -> bool:
    """The cost-balanced ranges are used unless RF_ATTN_SCHED=0 or the one-wave-per-SIMD kernel runs (attn_schedule)."""
    return os.environ.get("RF_ATTN_SCHED", "1") != "0" and os.environ.get("RF_ATTN_P4") != "1"


def attn_schedule(problems, n_heads: int, device) -> Optional[torch.Tensor]:
    """Device copy of the cost-balanced ranges for `problems` (host [P, 5] list/array), built once per plan;
    None when RF_ATTN_SCHED=0 (equal tile counts per workgroup, for A/B), and under RF_ATTN_P4=1: the schedule
    prices the 8-wave kernel's merge order (last partial first, publish deferred to the next prologue), which the
    one-wave-per-SIMD kernel does not share, so it runs on the equal split of each XCD group instead."""
    if not attn_schedule_enabled():
        return None
    return torch.from_numpy(attn_schedule_host(problems, n_heads, attn_grid(device))).to(device)


def rope_pair_perm(dim: int) -> torch.Tensor:
    """Row permutation of a q or k projection (dim = heads * 128) for gemm_qk_rope: per head, new row 2 m + t is old
    row m + 64 t (the rotate-half pairs (m, m + 64) of rope.py side by side, so one lane's 4 output columns hold
    two whole pairs).  Apply the same permutation to q and k (q.k unchanged) and to their norm weights."""
    _check(dim % 128 == 0, "rope_pair_perm: dim must be a multiple of 128")
    m = torch.arange(64)
    head = torch.stack([m, m + 64], dim=1).reshape(-1)  # [0, 64, 1, 65, ...]
    return (torch.arange(dim // 128)[:, None] * 128 + head[None, :]).reshape(-1)


def gemm_qk_rope(xg: torch.Tensor, w: torch.Tensor, out: torch.Tensor, ss: Optional[torch.Tensor], eps: float,
                 seg_w: int, n_seg: int, norm_w: Optional[torch.Tensor], seg_ss: Optional[torch.Tensor],
                 pos: Optional[torch.Tensor], freqs: Optional[torch.Tensor], q_scale: float = 1.0,
                 tag: Optional[str] = None, pos_div: int = 1) -> torch.Tensor:
    """rf_gemm_qk_rope: out (bf16) = the q/k(/v) projection of the deferred-norm operand xg (1 / rms(x) from ss, as
    gemm_rownorm) with, on its first n_seg segments of seg_w columns (rows of w permuted by rope_pair_perm),
    rope(norm_w * y) written (segment 0 also times q_scale) and seg_ss [M, n_seg, 8] = partial sums of y^2 when
    norm_w is given (the q/k norm's 1 / rms: row_rms_scale for k, attention(q_ss=...) for q)."""
    _check(xg.dtype in HALF and w.dtype == xg.dtype, "gemm_qk_rope: xg / w must both be bf16 or both fp16")
    _dev(xg, xg.dtype, "xg")
    _dev(w, w.dtype, "w")
    _dev(out, torch.bfloat16, "out")
    m, k = xg.shape
    n, k2 = w.shape
    _check(k == k2 and out.shape[0] == m and out.shape[1] >= n, "gemm_qk_rope: shape mismatch")
    if ss is not None:
        _dev(ss, torch.float32, "ss")
        _check(ss.shape[0] >= m and ss.shape[1] == PRENORM_SLOTS and ss.is_contiguous(), "gemm_qk_rope: ss shape")
    if norm_w is not None:
        _dev(norm_w, torch.float32, "norm_w")
        _check(norm_w.numel() == n_seg * seg_w, "gemm_qk_rope: norm_w size")
        _dev(seg_ss, torch.float32, "seg_ss")
        _check(seg_ss.is_contiguous() and seg_ss.shape[0] >= m and seg_ss.shape[1:] == (n_seg, PRENORM_SLOTS),
               "gemm_qk_rope: seg_ss [M, n_seg, 8]")
    if pos is not None:
        _dev(pos, torch.float32, "pos")
        _check(pos.shape[0] >= (m + pos_div - 1) // pos_div and pos.shape[1] >= 9 and freqs is not None,
               "gemm_qk_rope: pos [M / pos_div, 9] with freqs")
    ws = _gemm_workspace(xg.device)
    _t0(tag)
    call("rf_gemm_qk_rope", ptr(xg), xg.stride(0), ptr(w), w.stride(0), ptr(out), out.stride(0), m, n, k, ptr(ss),
         k, eps, ptr(seg_ss) if norm_w is not None else None, seg_w, n_seg, ptr(norm_w), ptr(pos),
         pos.stride(0) if pos is not None else 0, pos_div, ptr(freqs), freqs.numel() if (pos is not None) else 0,
         float(q_scale), _dt(xg), ptr(ws), ws.numel(), stream())
    return out


def row_rms_scale(x: torch.Tensor, ss: torch.Tensor, eps: float, scale: float = 1.0) -> torch.Tensor:
    """rf_row_rms_scale: x (bf16 rows, in place) *= scale / sqrt(sum(ss[r, :8]) / x.shape[1] + eps); ss a float view
    whose rows hold the 8 partial sums (e.g. seg_ss[:, 1] for the k segment)."""
    _dev(x, torch.bfloat16, "x")
    _check(ss.dtype == torch.float32 and ss.device == x.device and ss.shape[0] >= x.shape[0]
           and ss.shape[-1] == PRENORM_SLOTS and ss.stride(-1) == 1, "row_rms_scale: ss rows of 8 partial sums")
    call("rf_row_rms_scale", ptr(x), x.stride(0), x.shape[0], x.shape[1], ptr(ss), ss.stride(0), eps, float(scale),
         stream())
    return x


def attention(q, k, v, out, problems: torch.Tensor, max_q_len: int, n_heads: int,
              scale: Optional[float] = None, tag: Optional[str] = None, max_k_len: Optional[int] = None,
              n_split: Optional[int] = None, q_prescaled: bool = False,
              schedule: Optional[torch.Tensor] = None, q_ss: Optional[torch.Tensor] = None,
              q_eps: float = 0.0) -> torch.Tensor:
    """Varlen attention; problems int32 [P, 5] = (q_start, q_len, k_start, k_len, v_start).

    n_split None/0: the stream-K kernel (balanced over the CUs, cut units merged in-kernel), with the
    workgroup ranges of `schedule` (attn_schedule of the same problems and heads) when given;
    n_split >= 1: the legacy per-unit kernel with flash-decoding splits + rf_attn_combine.
    q_prescaled: q already carries scale*log2(e) (qk_norm_rope q_scale=Q_LOG2_SCALE).  q/k/v are bf16 or
    all fp16 (rf_attn_fwd_dt: the fp16 operands the reference's default half precision hands flash_attn; the
    stream-K kernel only).  q_ss (rf_attn_fwd_qn; bf16, the stream-K kernel): rows of 8 partial sums of squares of
    q before its norm (gemm_qk_rope's seg_ss[:, 0]): q rows are scaled by Q_LOG2_SCALE / rms as they load
    (q_prescaled implied)."""
    _check(q.dtype in HALF, f"attention: q/k/v must be bf16 or fp16, got {q.dtype}")
    if q_ss is not None:
        _check(q.dtype == torch.bfloat16 and scale is None and (n_split is None or n_split == 0),
               "attention: q_ss needs bf16 q/k/v on the stream-K kernel")
        _check(q_ss.dtype == torch.float32 and q_ss.shape[-1] == PRENORM_SLOTS and q_ss.stride(-1) == 1
               and q_ss.shape[0] >= q.shape[0], "attention: q_ss rows of 8 partial sums")
        _dev(problems, torch.int32, "problems")
        _dev(out, out.dtype, "out")
        if schedule is not None:
            _dev(schedule, torch.int64, "schedule")
        ws = _attn_workspace(out.device)
        _t0(tag)
        call("rf_attn_fwd_qn", ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0), ptr(out), out.stride(0),
             DT_F16 if out.dtype == torch.float16 else DT_BF16, ptr(q_ss), q_ss.stride(0), q.shape[1], q_eps,
             Q_LOG2_SCALE, ptr(problems), problems.shape[0], n_heads, q.shape[1] // n_heads, ptr(ws), ptr(schedule),
             schedule.numel() - 1 if schedule is not None else 0, stream())
        return out
    for t, nme in ((q, "q"), (k, "k"), (v, "v")):
        _dev(t, q.dtype, nme)
    _check(out.dtype in HALF, "attention: out must be bf16 or fp16")
    _dev(out, out.dtype, "out")
    _dev(problems, torch.int32, "problems")
    _check(problems.dim() == 2 and problems.shape[1] == 5, "attention: problems must be [P, 5]")
    hd = q.shape[1] // n_heads
    if q_prescaled:
        _check(scale is None, "attention: q_prescaled implies the scale")
        scale = LN2
    scale = 1.0 / math.sqrt(hd) if scale is None else scale
    if n_split is None:
        env = os.environ.get("RF_ATTN_SPLIT")
        n_split = int(env) if env else 0
    ws, rows = None, out.shape[0]
    if n_split == 0:
        ws = _attn_workspace(out.device)
    elif n_split > 1:
        nbytes = load().rf_attn_workspace_bytes(rows, n_heads, n_split)
        ws = torch.empty(nbytes // 4, dtype=torch.float32, device=out.device)
    _t0(tag)
    if n_split == 0:
        if schedule is not None:
            _dev(schedule, torch.int64, "schedule")
        call("rf_attn_fwd_dt", ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0), ptr(out),
             out.stride(0), DT_F16 if q.dtype == torch.float16 else DT_BF16,
             DT_F16 if out.dtype == torch.float16 else DT_BF16, ptr(problems), problems.shape[0],
             n_heads, hd, scale, ptr(ws), ptr(schedule), schedule.numel() - 1 if schedule is not None else 0,
             stream())
        return out
    _check(q.dtype == torch.bfloat16 and out.dtype == torch.bfloat16, "attention: the legacy split kernels are bf16")
    call("rf_attn_fwd", ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0), ptr(out), out.stride(0),
         ptr(problems), problems.shape[0], max_q_len, n_heads, hd, scale, n_split, ptr(ws), rows, stream())
    if n_split > 1:
        call("rf_attn_combine", ptr(ws), rows, n_split, n_heads, None, rows, ptr(out), out.stride(0), stream())
    return out


def encoder_layers(layers, qk_norm: bool):
    """Host array of rf_encoder_layer (device pointers) for the encoder stack's weights (model._Layer objects with
    query_norm, w_in, qk_norm, w_out, ffn_norm, w13, w2).  The caller keeps the tensors alive."""
    from ._lib import EncoderLayer
    arr = (EncoderLayer * len(layers))()
    for e, L in zip(arr, layers):
        e.attn_norm, e.w_qkv, e.w_out = ptr(L.query_norm), ptr(L.w_in), ptr(L.w_out)
        e.qk_norm = ptr(L.qk_norm) if qk_norm else None
        e.ffn_norm, e.w13, e.w2 = ptr(L.ffn_norm), ptr(L.w13), ptr(L.w2)
    return arr


def encoder_forward(x: torch.Tensor, layers, n_layers: int, n_heads: int, ffn_dim: int, operands: torch.dtype,
                    eps: float, pos: Optional[torch.Tensor], freqs: Optional[torch.Tensor], problems: torch.Tensor,
                    schedule: Optional[torch.Tensor] = None, tag: Optional[str] = None,
                    qk_fused: bool = False) -> torch.Tensor:
    """x [T, D] f32 through the whole encoder stack in place, one C call (rf_encoder_forward; `layers` from
    encoder_layers).  Same launches, same order and so the same bits as the per-op sequence of model._stage1.
    qk_fused: the layers' q/k weights are in rope_pair_perm order (the fused QK path, rf.h ABI 16)."""
    from ._lib import EncoderDesc
    import ctypes
    _dev(x, torch.float32, "x")
    _check(operands in HALF, "encoder_forward: operands must be bf16 or fp16")
    _dev(problems, torch.int32, "problems")
    rows, dim = x.shape
    _check(dim == n_heads * 128, "encoder_forward: dim must be n_heads * 128")
    if pos is not None:
        _dev(pos, torch.float32, "pos")
        _check(pos.shape[0] >= rows and pos.shape[1] == 9 and freqs is not None, "encoder_forward: pos [T, 9] + freqs")
    if schedule is not None:
        _dev(schedule, torch.int64, "schedule")
    odt = DT_F16 if operands == torch.float16 else DT_BF16
    lib = load()
    ws = torch.empty(int(lib.rf_encoder_workspace_bytes(rows, dim, ffn_dim, odt)), dtype=torch.uint8, device=x.device)
    gws = _gemm_workspace(x.device)
    d = EncoderDesc(n_layers=n_layers, rows=rows, dim=dim, n_heads=n_heads, ffn_dim=ffn_dim, operand_dtype=odt, eps=eps,
                    layers=ctypes.addressof(layers), pos=ptr(pos), ld_pos=pos.stride(0) if pos is not None else 0,
                    freqs=ptr(freqs), n_freqs=freqs.numel() if freqs is not None else 0, problems=ptr(problems),
                    n_problems=problems.shape[0], bounds=ptr(schedule),
                    grid=schedule.numel() - 1 if schedule is not None else 0, workspace=ptr(ws), gemm_ws=ptr(gws),
                    gemm_ws_bytes=gws.numel(), attn_ws=ptr(_attn_workspace(x.device)),
                    timer_attn=int(_timer_takes(tag, n_layers)), qk_fused=int(qk_fused))
    call("rf_encoder_forward", ptr(x), x.stride(0), ctypes.addressof(d), stream())
    return x


def decoder_layers(layers, qk_norm: bool):
    """Host array of rf_decoder_layer (device pointers) for the decoder stack's weights (model._Layer objects)."""
    from ._lib import DecoderLayer
    arr = (DecoderLayer * len(layers))()
    for e, L in zip(arr, layers):
        e.query_norm, e.w_q, e.kv_norm, e.w_kv, e.w_out = (ptr(L.query_norm), ptr(L.wq), ptr(L.kv_norm), ptr(L.wkv),
                                                           ptr(L.wo))
        e.q_norm = ptr(L.q_norm) if qk_norm else None
        e.k_norm = ptr(L.k_norm) if qk_norm else None
        if hasattr(L, "ws_in"):
            e.self_norm, e.w_self_in, e.w_self_out = ptr(L.self_norm), ptr(L.ws_in), ptr(L.ws_out)
            e.self_qk_norm = ptr(L.sqk_norm) if qk_norm else None
        e.ffn_norm, e.w13, e.w2 = ptr(L.ffn_norm), ptr(L.w13), ptr(L.w2)
    return arr


def decoder_forward(x: torch.Tensor, layers, n_layers: int, n_heads: int, ffn_dim: int, operands: torch.dtype,
                    eps: float, ctx: torch.Tensor, kv: dict, cross: dict, self_attn: dict, taps=(),
                    tag: Optional[str] = None) -> torch.Tensor:
    """x [T2, D] f32 through the whole decoder stack in place, one C call (rf_decoder_forward; `layers` from
    decoder_layers).  kv: ctx_norm, w_kv_all (None = per-layer K/V), k_batch, k_norm_all, kv_src_rows, kv_pos,
    freqs; cross: ray_pos, ray_pos_div, problems, schedule, qk_fused (the q/k weights in rope_pair_perm order: the
    query rotation in its projection's epilogue); self_attn: swin, n_images, grid_h, grid_w, window, shift,
    problems; taps: (layer, planes_hi, planes_lo or None, ld) in layer order."""
    from ._lib import DecoderDesc, DecoderTap
    import ctypes
    _dev(x, torch.float32, "x")
    _dev(ctx, torch.float32, "ctx")
    _check(operands in HALF, "decoder_forward: operands must be bf16 or fp16")
    rows, dim = x.shape
    _check(dim == n_heads * 128, "decoder_forward: dim must be n_heads * 128")
    _dev(cross["problems"], torch.int32, "cross problems")
    _dev(kv["kv_src_rows"], torch.int32, "kv_src_rows")
    for key in ("kv_pos", "freqs"):
        if kv.get(key) is not None:
            _dev(kv[key], torch.float32, key)
    if cross.get("ray_pos") is not None:
        _dev(cross["ray_pos"], torch.float32, "ray_pos")
    if cross.get("schedule") is not None:
        _dev(cross["schedule"], torch.int64, "schedule")
    tarr = (DecoderTap * max(1, len(taps)))()
    for e, (layer, hi, lo, ld) in zip(tarr, taps):
        e.layer, e.p_hi, e.p_lo, e.p_ld = layer, ptr(hi), ptr(lo), ld
    gws = _gemm_workspace(x.device)
    sch = cross.get("schedule")
    pos, rpos, freqs = kv.get("kv_pos"), cross.get("ray_pos"), kv.get("freqs")
    sp = self_attn.get("problems")
    d = DecoderDesc(n_layers=n_layers, rows=rows, dim=dim, n_heads=n_heads, ffn_dim=ffn_dim,
                    operand_dtype=DT_F16 if operands == torch.float16 else DT_BF16, eps=eps,
                    layers=ctypes.addressof(layers), ctx=ptr(ctx), ld_ctx=ctx.stride(0), ctx_rows=ctx.shape[0],
                    ctx_dim=ctx.shape[1], ctx_norm=ptr(kv.get("ctx_norm")), w_kv_all=ptr(kv.get("w_kv_all")),
                    kv_rows=kv["kv_src_rows"].numel(), kv_src_rows=ptr(kv["kv_src_rows"]), kv_pos=ptr(pos),
                    ld_kv_pos=pos.stride(0) if pos is not None else 0, k_batch=int(bool(kv.get("k_batch"))),
                    k_norm_all=ptr(kv.get("k_norm_all")), freqs=ptr(freqs),
                    n_freqs=freqs.numel() if freqs is not None else 0, ray_pos=ptr(rpos),
                    ld_ray_pos=rpos.stride(0) if rpos is not None else 0, ray_pos_div=cross.get("ray_pos_div", 1),
                    cross_problems=ptr(cross["problems"]), n_cross=cross["problems"].shape[0], cross_bounds=ptr(sch),
                    cross_grid=sch.numel() - 1 if sch is not None else 0, swin=int(bool(self_attn.get("swin"))),
                    n_images=self_attn.get("n_images", 0), grid_h=self_attn.get("grid_h", 0),
                    grid_w=self_attn.get("grid_w", 0), window=self_attn.get("window", 0),
                    shift=self_attn.get("shift", 0), self_problems=ptr(sp), n_self=sp.shape[0] if sp is not None else 0,
                    taps=ctypes.addressof(tarr), n_taps=len(taps), gemm_ws=ptr(gws), gemm_ws_bytes=gws.numel(),
                    attn_ws=ptr(_attn_workspace(x.device)))
    lib = load()
    ws = torch.empty(int(lib.rf_decoder_workspace_bytes(ctypes.addressof(d))), dtype=torch.uint8, device=x.device)
    d.workspace = ptr(ws)
    d.timer_cross = int(_timer_takes(tag, n_layers))
    d.qk_fused = int(bool(cross.get("qk_fused")))
    call("rf_decoder_forward", ptr(x), x.stride(0), ctypes.addressof(d), stream())
    return x


def swin_attention(q, k, v, out, n_images: int, grid_h: int, grid_w: int, shift: int, n_heads: int,
                   window: int = 8, q_prescaled: bool = False, qk_norm=None) -> torch.Tensor:
    """Shifted-window self-attention (rf_swin_attn_fwd_dt).  ``qk_norm = (qk_ss, norm_w, eps)`` folds the full-width
    q/k RMSNorm (and the softmax scale on q) into the kernel's loads (rf_swin_attn_fwd_qkn): q, k as the projection
    wrote them, qk_ss [rows, 2, PRENORM_SLOTS] from gemm_rownorm(seg_ss=..., seg_w=D), norm_w [2D] (required)."""
    for t, nme in ((q, "q"), (k, "k"), (v, "v")):
        _dev(t, torch.bfloat16, nme)
    _check(out.dtype in HALF, "swin_attention: out must be bf16 or fp16")
    _dev(out, out.dtype, "out")
    hd = q.shape[1] // n_heads
    odt = DT_F16 if out.dtype == torch.float16 else DT_BF16
    if qk_norm is None:
        call("rf_swin_attn_fwd_dt", ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0), ptr(out),
             out.stride(0), odt, n_images, grid_h, grid_w, window, shift, n_heads, hd,
             LN2 if q_prescaled else 1.0 / math.sqrt(hd), stream())
        return out
    qk_ss, norm_w, eps = qk_norm
    _dev(qk_ss, torch.float32, "qk_ss")
    _check(qk_ss.is_contiguous() and qk_ss.shape[1:] == (2, PRENORM_SLOTS), "swin_attention: qk_ss [rows, 2, 8]")
    call("rf_swin_attn_fwd_qkn", ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0), ptr(out),
         out.stride(0), odt, n_images, grid_h, grid_w, window, shift, n_heads, hd, LN2, ptr(qk_ss), ptr(norm_w), eps,
         Q_LOG2_SCALE, stream())
    return out


def texture_pack(texture: torch.Tensor, log_channels: int, dst_row: torch.Tensor, out: torch.Tensor):
    _dev(texture, torch.float32, "texture")
    _check(texture.is_contiguous(), "texture must be contiguous")
    b, n, c = texture.shape[:3]
    pe = texture[0, 0, 0].numel() if texture.dim() > 3 else 1
    call("rf_texture_pack", ptr(texture), b * n, c, pe, log_channels, ptr(dst_row), ptr(out), out.stride(0), stream())
    return out


def texture_pack_if(flag: torch.Tensor, texture: torch.Tensor, log_channels: int, dst_row: torch.Tensor,
                    out: torch.Tensor):
    """texture_pack that runs only when the device flag is non-zero (the general texture path)."""
    _dev(flag, torch.int32, "flag")
    _dev(texture, torch.float32, "texture")
    _check(texture.is_contiguous(), "texture must be contiguous")
    b, n, c = texture.shape[:3]
    pe = texture[0, 0, 0].numel() if texture.dim() > 3 else 1
    call("rf_texture_pack_if", ptr(flag), ptr(texture), b * n, c, pe, log_channels, ptr(dst_row), ptr(out),
         out.stride(0), stream())
    return out


def texture_scan(texture: torch.Tensor, log_channels: int, dst_row: torch.Tensor, coef: torch.Tensor,
                 flag: torch.Tensor, flag_clear: Optional[torch.Tensor] = None):
    """In-place log encode + per-row channel constants of to_h5-format textures; flag = 1 if any valid row is
    not of that form.  Without flag_clear (rf_texture_scan) the flag is reset first by a memset; with it
    (rf_texture_scan2) flag must already be 0 and the kernel zeroes flag_clear instead (frame-parity flags)."""
    _dev(texture, torch.float32, "texture")
    _dev(coef, torch.float32, "coef")
    _dev(flag, torch.int32, "flag")
    _check(texture.is_contiguous() and texture.dim() == 5 and tuple(texture.shape[3:]) == (32, 32),
           "texture_scan: texture must be contiguous [B, N, C, 32, 32]")
    b, n, c = texture.shape[:3]
    if flag_clear is not None:
        _dev(flag_clear, torch.int32, "flag_clear")
        call("rf_texture_scan2", ptr(texture), b * n, c, 32 * 32, log_channels, ptr(dst_row), ptr(coef),
             coef.stride(0), ptr(flag), ptr(flag_clear), stream())
        return coef
    call("rf_texture_scan", ptr(texture), b * n, c, 32 * 32, log_channels, ptr(dst_row), ptr(coef), coef.stride(0),
         ptr(flag), stream())
    return coef


def texture_linear(coef: torch.Tensor, wsum: torch.Tensor, bias: Optional[torch.Tensor], out: torch.Tensor,
                   flag: torch.Tensor):
    """out = bias + coef @ wsum when the device flag is 0 (rf_texture_linear)."""
    _dev(coef, torch.float32, "coef")
    _dev(wsum, torch.float32, "wsum")
    _dev(out, torch.float32, "out")
    _dev(flag, torch.int32, "flag")
    ch, n = wsum.shape
    _check(coef.shape[1] >= ch and out.shape == (coef.shape[0], n) and wsum.is_contiguous(),
           "texture_linear: shape mismatch")
    if bias is not None:
        _dev(bias, torch.float32, "bias")
    call("rf_texture_linear", ptr(coef), coef.stride(0), out.shape[0], ch, ptr(wsum), ptr(bias), ptr(out),
         out.stride(0), n, ptr(flag), stream())
    return out


def _dt(out: torch.Tensor) -> int:
    _check(out.dtype in HALF, "16-bit output must be bf16 or fp16")
    return DT_F16 if out.dtype == torch.float16 else DT_BF16


def vn_encode(vn: torch.Tensor, dst_row: torch.Tensor, n_freqs: int, out: torch.Tensor):
    _dev(vn, torch.float32, "vn")
    _check(vn.is_contiguous() and vn.shape[-1] == 9, "vn must be contiguous [..., 9]")
    call("rf_vn_encode_dt", ptr(vn), vn.numel() // 9, ptr(dst_row), n_freqs, ptr(out), out.stride(0), _dt(out),
         stream())
    return out


def ray_tokens(c2w: torch.Tensor, fov_deg: torch.Tensor, res: int, patch: int, out: torch.Tensor,
               ray_pos: torch.Tensor):
    _dev(c2w, torch.float32, "c2w")
    _check(c2w.is_contiguous() and fov_deg.is_contiguous(), "c2w/fov must be contiguous")
    call("rf_ray_tokens_dt", ptr(c2w), ptr(fov_deg), c2w.numel() // 16, res, patch, ptr(out), ptr(ray_pos), _dt(out),
         stream())
    return out


def patchify_rays(rays_d: torch.Tensor, patch: int, out: torch.Tensor):
    _dev(rays_d, torch.float32, "rays_d")
    _check(rays_d.is_contiguous() and rays_d.shape[-1] == 3 and rays_d.shape[-2] == rays_d.shape[-3],
           "rays_d must be contiguous [*, res, res, 3]")
    res = rays_d.shape[-2]
    call("rf_patchify_rays_dt", ptr(rays_d), rays_d.numel() // (res * res * 3), res, patch, ptr(out), _dt(out),
         stream())
    return out


def scene_pos(tris: torch.Tensor, valid_idx, scene_off, c2w: Optional[torch.Tensor], n_scenes: int, n_views: int,
              n_reg: int, pos_out: torch.Tensor, set_off: torch.Tensor, max_tris: int):
    """Triangle RoPE positions + register-token centres (rf_scene_pos; max_tris >= every scene's valid count)."""
    _dev(tris, torch.float32, "tris")
    _check(tris.is_contiguous(), "tris must be contiguous")
    sets = n_scenes * n_views if c2w is not None else n_scenes
    nparts = int(load().rf_scene_pos_partials(sets, max_tris))
    parts = torch.empty(max(nparts, 1), dtype=torch.float32, device=pos_out.device)
    call("rf_scene_pos", ptr(tris), ptr(valid_idx), ptr(scene_off), ptr(c2w), n_scenes, n_views, n_reg, ptr(pos_out),
         ptr(set_off), max_tris, ptr(parts), parts.numel(), stream())
    return pos_out


def embed(out: torch.Tensor, out_rows: Optional[torch.Tensor], rows: int, base: Optional[torch.Tensor],
          base_rows: int, in0=None, w0=None, eps0: float = FLT_EPS, in1=None, w1=None, eps1: float = FLT_EPS):
    _dev(out, torch.float32, "out")
    dim = out.shape[1]
    call("rf_embed", ptr(out), out.stride(0), ptr(out_rows), rows, dim, ptr(base), base_rows, ptr(in0),
         in0.stride(0) if in0 is not None else 0, ptr(w0), eps0, ptr(in1), in1.stride(0) if in1 is not None else 0,
         ptr(w1), eps1, stream())
    return out


def hdr_output(logits: torch.Tensor, out: torch.Tensor, elu_alpha: float, log_decode: bool,
               channels_last: bool = True):
    _dev(logits, torch.float32, "logits")
    _check(logits.is_contiguous() and out.is_contiguous(), "hdr_output: contiguous tensors required")
    n, c, h, w = logits.shape
    call("rf_hdr_output", ptr(logits), ptr(out), n, c, h, w, elu_alpha, int(log_decode), int(channels_last), stream())
    return out
