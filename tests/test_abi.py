"""The C-ABI library loads and exports every symbol include/rf.h declares (no GPU needed)."""
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    text = open(os.path.join(REPO, "include", "rf.h")).read()
    return sorted(set(re.findall(r"^(?:int|int64_t|const char\*)\s+(rf_\w+)\(", text, flags=re.M)))


def test_header_lists_entry_points():
    fns = header_functions()
    assert "rf_gemm_bf16" in fns and "rf_attn_fwd" in fns and len(fns) >= 14


def test_library_exports_every_header_symbol():
    import torch  # noqa: F401
    from renderformer_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("librfhip.so not built (run __graft_entry__.build())")
    lib = _lib.load(require_device=False)
    for fn in header_functions():
        assert hasattr(lib, fn), fn
    assert lib.rf_abi_version() == 16
    # every int-returning entry point has a ctypes signature in the binding
    assert set(_lib.SIGNATURES) == set(header_functions()) - {"rf_last_error", "rf_abi_version", "rf_build_flags",
                                                               "rf_attn_workspace_bytes", "rf_gemm_workspace_bytes",
                                                               "rf_scene_pos_partials", "rf_attn_grid",
                                                               "rf_encoder_workspace_bytes",
                                                               "rf_decoder_workspace_bytes"}
    # the production build (what the product path loads) carries no study kernels; the study build says so
    assert lib.rf_build_flags() in (0, 1)


def test_invalid_arguments_raise_value_error_without_device():
    """Argument validation happens before any launch, so it is testable on CPU."""
    import ctypes
    import torch  # noqa: F401
    from renderformer_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("librfhip.so not built")
    lib = _lib.load(require_device=False)
    rc = lib.rf_gemm_bf16(ctypes.c_void_p(16), 64, ctypes.c_void_p(16), 64, ctypes.c_void_p(16), 128, None,
                          10, 100, 64, 0, None, 0, None)  # N % 128 != 0
    assert rc == 1 and b"multiple of 128" in lib.rf_last_error()
    rc = lib.rf_attn_fwd(ctypes.c_void_p(16), 256, ctypes.c_void_p(16), 256, ctypes.c_void_p(16), 256,
                         ctypes.c_void_p(16), 256, ctypes.c_void_p(16), 1, 10, 2, 64, 1.0, 1, None, 0, None)
    assert rc == 1 and b"head_dim" in lib.rf_last_error()


@pytest.mark.gpu
def test_device_error_word_surfaces_on_next_call():
    """A device-side error (here raised on purpose by a debug kernel; in production a stream-K owner whose
    partner never published) makes the next entry point fail loudly, without a device sync, until cleared."""
    import torch
    from renderformer_amd import _lib, ops
    lib = _lib.load()
    assert lib.rf_device_error() == 0
    _lib.call("rf_debug_raise_device_error", 7, _lib.stream())
    torch.cuda.synchronize()
    assert lib.rf_device_error() == 7
    x = torch.randn(4, 256, device="cuda")
    out = torch.empty(4, 256, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(_lib.DeviceError, match="device error 7"):
        ops.rmsnorm(x, torch.ones(256, device="cuda"), 1e-6, out)
    lib.rf_clear_device_error()
    ops.rmsnorm(x, torch.ones(256, device="cuda"), 1e-6, out)  # clean again


@pytest.mark.gpu
def test_kernel_timer_times_the_tagged_launch():
    """rf_ktimer_arm + a tagged op: exactly the tagged launch is timed (dispatch-packet events), its duration is
    positive and no longer than a marker-event bracket around the same launch."""
    import torch
    from renderformer_amd import ops
    a = torch.randn(4096, 1024, device="cuda").bfloat16()
    w = torch.randn(8192, 1024, device="cuda").bfloat16()
    out = torch.empty(4096, 8192, device="cuda", dtype=torch.bfloat16)
    ops.gemm(a, w, out)  # warm
    t = ops.KernelTimer("timed")
    ops.TIMER = t
    try:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.gemm(a, w, out, tag="timed")
        e1.record()
        ops.gemm(a, w, out, tag="other")  # not timed
        ops.gemm(a, w, out, tag="timed")
    finally:
        ops.TIMER = None
    d = t.durations_ms()
    torch.cuda.synchronize()
    assert len(d) == 2 and all(x > 0 for x in d), d
    assert d[0] <= e0.elapsed_time(e1) + 1e-3
    assert t.durations_ms() == []  # pairs released


def _sk_pieces(bounds, units):
    """(workgroup, first tile, end tile, unit start, unit end) of every piece of a stream-K range table"""
    out = []
    for w in range(len(bounds) - 1):
        x = int(bounds[w])
        while x < bounds[w + 1]:
            us, ue = next((a, b) for a, b in units if a <= x < b)
            e = min(int(bounds[w + 1]), ue)
            out.append((w, x, e, us, ue))
            x = e
    return out


@pytest.mark.parametrize("probs,grid", [
    ([[0, 5649, 0, 5649, 0]], 256),                                   # stage 1 at the bench shape
    ([[0, 4096, 0, 5649, 0]], 256),                                   # cross-attention, one view
    ([[0, 5649, 0, 5649, 0], [5649, 3000, 5649, 3000, 5649]], 256),   # two scenes, ragged
    ([[0, 0, 0, 0, 0], [0, 300, 0, 70, 0], [300, 40, 70, 1, 70]], 64),  # empty problem, tiny ones
    ([[0, 100, 0, 100, 0]], 512),                                      # fewer tiles than workgroups
])
def test_attn_schedule_covers_every_tile_once(probs, grid):
    """rf_attn_schedule (host only): monotone bounds from 0 to the total tile count, so every tile of the
    flattened (problem, head, 256-row block, 64-key tile) space belongs to exactly one workgroup, and each unit's
    pieces are consecutive workgroups (the kernel's owner walks workgroups wg+1.. until the unit ends)."""
    import numpy as np
    import torch  # noqa: F401
    from renderformer_amd import _lib, ops
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("librfhip.so not built")
    H = 8
    b = ops.attn_schedule_host(probs, H, grid)
    units, tot = [], 0
    for q0, ql, k0, kl, v0 in probs:
        nt = (kl + 63) // 64
        n_units = H * ((ql + 255) // 256) if ql > 0 else 0
        for _ in range(n_units if nt else 0):
            units.append((tot, tot + nt))
            tot += nt
    assert b.shape == (grid + 1,) and b[0] == 0 and b[-1] == tot
    assert np.all(np.diff(b) >= 0)
    pieces = _sk_pieces(b, units)
    assert sum(e - x for _, x, e, _, _ in pieces) == tot
    by_unit = {}
    for w, x, e, us, ue in pieces:
        by_unit.setdefault(us, []).append(w)
    for ws in by_unit.values():
        assert ws == list(range(ws[0], ws[0] + len(ws)))


def _sk_logical(nwg, units):
    """Python mirror of common.h SkLayout: logical index of every blockIdx, and the groups' logical spans."""
    nx = min(8, nwg)
    G = max(1, units) if units < nx else nx
    cnt = [(nwg - x + nx - 1) // nx for x in range(nx)]
    xlo = [(g * nx + G - 1) // G for g in range(G + 1)]
    base = [sum(cnt[:xlo[g]]) for g in range(G + 1)]
    logical = {}
    for hw in range(nwg):
        x = hw % nx
        g = x * G // nx
        rank = sum(1 for y in range(xlo[g], xlo[g + 1]) for j in range(cnt[y]) if nx * j + y > hw)
        logical[hw] = base[g] + rank
    assert sorted(logical.values()) == list(range(nwg))  # a bijection
    return logical, [(base[g], base[g + 1]) for g in range(G)]


@pytest.mark.parametrize("probs,grid", [
    ([[0, 5649, 0, 5649, 0]], 256),                                   # stage 1, bench shape (23 units per group)
    ([[0, 4096, 0, 5649, 0]], 256),                                   # cross-attention, one view (2-way cuts)
    ([[0, 6225, 0, 6225, 0], [6225, 11819, 6225, 11819, 6225]], 256),  # bunny + lucy sized scenes in one launch
    ([[0, 5649, 0, 5649, 0]], 100),                                   # grid not a multiple of 8
    ([[0, 700, 0, 900, 0]], 256),                                     # fewer units than groups
])
def test_attn_schedule_forward_progress(probs, grid):
    """Every owner (the block holding a unit's first tile, which merges the unit's other pieces) has a HIGHER
    blockIdx than every block it waits on, and a unit never spans two XCD groups: the waits only go to
    earlier-dispatched blocks, so the launch drains with no co-residency assumption (common.h SkLayout)."""
    import numpy as np
    import torch  # noqa: F401
    from renderformer_amd import _lib, ops
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("librfhip.so not built")
    H = 8
    b = ops.attn_schedule_host(probs, H, grid)
    units, tot = [], 0
    for q0, ql, k0, kl, v0 in probs:
        nt = (kl + 63) // 64
        for _ in range(H * ((ql + 255) // 256) if nt and ql else 0):
            units.append((tot, tot + nt))
            tot += nt
    assert b[0] == 0 and b[-1] == tot and np.all(np.diff(b) >= 0)
    logical, spans = _sk_logical(grid, len(units))
    hw_of = {L: hw for hw, L in logical.items()}
    group_of = {L: g for g, (s, e) in enumerate(spans) for L in range(s, e)}
    by_unit = {}
    for w, x, e, us, ue in _sk_pieces(b, units):
        by_unit.setdefault(us, []).append(w)
    cut = 0
    for ws in by_unit.values():
        assert len({group_of[w] for w in ws}) == 1, ws        # one group per unit
        owner = ws[0]
        assert all(hw_of[owner] > hw_of[w] for w in ws[1:])    # owner waits only on lower blockIdx
        cut += len(ws) > 1
    if probs == [[0, 5649, 0, 5649, 0]] and grid == 256:
        assert cut == 184  # every unit (89 tiles) is longer than a workgroup's share (64): all are cut


def test_attn_schedule_balances_the_bench_shape():
    """At the stage-1 bench shape the balanced table gives the workgroups that hold a single piece ("mid": one
    prologue, one publish) more tiles than those with two pieces, and no workgroup is left empty."""
    import numpy as np
    import torch  # noqa: F401
    from renderformer_amd import _lib, ops
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("librfhip.so not built")
    b = ops.attn_schedule_host([[0, 5649, 0, 5649, 0]], 8, 256)
    d = np.diff(b)
    assert d.min() > 0
    units = [(89 * u, 89 * u + 89) for u in range(184)]
    pieces = _sk_pieces(b, units)
    per_wg = {}
    for w, *_ in pieces:
        per_wg[w] = per_wg.get(w, 0) + 1
    single = [d[w] for w in range(256) if per_wg[w] == 1]
    double = [d[w] for w in range(256) if per_wg[w] == 2]
    assert single and double and np.mean(single) > np.mean(double)


def _integration_binding_source():
    """The reference-side ctypes binding sketched in INTEGRATION.md (the first ```python block of section 2)."""
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    sec = text[text.index("## 2. C ABI"):]
    m = re.search(r"```python\n(.*?)```", sec, flags=re.S)
    assert m, "INTEGRATION.md section 2 lost its binding example"
    return m.group(1)


def test_integration_binding_parses():
    """The documented binding is valid Python that binds only symbols the header declares."""
    import ast
    src = _integration_binding_source()
    ast.parse(src)
    used = set(re.findall(r"_rf\.(rf_\w+)", src))
    assert used and used <= set(header_functions()) | {"rf_last_error"}, used - set(header_functions())


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["float16", "bfloat16"])
def test_integration_binding_runs_against_reference_attention(dtype):
    """Execute INTEGRATION.md's reference-side binding verbatim (only the library path filled in) the way the
    reference's attention switch would call it — flash_attn's qkv-packed varlen layout [T, 3, H, 128] with
    cu_seqlens (stage 1), and the kv-packed layout q [Tq, H, 128] / kv [Tk, 2, H, 128] with cu_seqlens_q /
    cu_seqlens_k (stage-2 cross-attention, attention.py:183-198) — against fp64 softmax attention, with the
    reference's default fp16 operands (torch_dtype=torch.float16, rendering_pipeline.py:37) and with bf16; the
    output keeps the input's type, and fp32 q/k/v are refused (as flash_attn refuses them)."""
    import math
    import torch
    from renderformer_amd import _lib
    dt = getattr(torch, dtype)
    tol = 2e-3 if dt == torch.float16 else 6e-3  # fp16 operands and P carry 3 more mantissa bits than bf16
    src = _integration_binding_source().replace('ctypes.CDLL("librfhip.so")', f'ctypes.CDLL({_lib.LIB_PATH!r})')
    ns = {}
    exec(compile(src, "INTEGRATION.md", "exec"), ns)
    H, hd = 4, 128
    lens = [300, 77, 1000]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device="cuda")
    T = sum(lens)
    g = torch.Generator(device="cpu").manual_seed(2)
    qkv = torch.randn(T, 3, H, hd, generator=g).to(dt).cuda()
    out = ns["rfhip_varlen_qkvpacked"](qkv, cu, max(lens))
    torch.cuda.synchronize()
    assert out.shape == (T, H, hd) and out.dtype == dt
    o = out.float().cpu()
    q, k, v = (qkv[:, i].double().cpu() for i in range(3))
    for a, b in zip(cu.tolist(), cu.tolist()[1:]):
        s = torch.einsum("qhd,khd->hqk", q[a:b], k[a:b]) / math.sqrt(hd)
        ref = torch.einsum("hqk,khd->qhd", torch.softmax(s, -1), v[a:b])
        err = ((o[a:b].double() - ref).norm() / ref.norm()).item()
        assert err < tol, (a, b, err)
    # the kv-packed binding: stage-2 cross-attention, 3 "views" of 256 rays over scenes of ragged lengths
    Hc, R = 8, 256
    klens = [700, 77, 1300]
    cuq = torch.arange(0, R * (len(klens) + 1), R, dtype=torch.int32, device="cuda")
    cuk = torch.tensor([0] + list(torch.tensor(klens).cumsum(0)), dtype=torch.int32, device="cuda")
    qc = torch.randn(R * len(klens), Hc, hd, generator=g).to(dt).cuda()
    kv = torch.randn(sum(klens), 2, Hc, hd, generator=g).to(dt).cuda()
    oc = ns["rfhip_varlen_kvpacked"](qc, kv, cuq, cuk, R, max(klens))
    torch.cuda.synchronize()
    assert oc.shape == qc.shape and oc.dtype == dt
    oc, qd, kd, vd = oc.float().cpu(), qc.double().cpu(), kv[:, 0].double().cpu(), kv[:, 1].double().cpu()
    for i in range(len(klens)):
        a, b, c0, c1 = cuq[i].item(), cuq[i + 1].item(), cuk[i].item(), cuk[i + 1].item()
        s = torch.einsum("qhd,khd->hqk", qd[a:b], kd[c0:c1]) / math.sqrt(hd)
        ref = torch.einsum("hqk,khd->qhd", torch.softmax(s, -1), vd[c0:c1])
        err = ((oc[a:b].double() - ref).norm() / ref.norm()).item()
        assert err < tol, (i, err)
    with pytest.raises(TypeError, match="fp16 and bf16"):
        ns["rfhip_varlen_qkvpacked"](qkv.float(), cu, max(lens))


def test_conv_desc_layout_matches_header(tmp_path):
    """dpt._ConvDesc (ctypes) has the size and field offsets of rf.h's rf_conv_desc (checked with the host C
    compiler on the header itself)."""
    import ctypes
    import shutil
    import subprocess
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no host C compiler")
    from renderformer_amd.dpt import _ConvDesc
    names = [f[0] for f in _ConvDesc._fields_]
    src = tmp_path / "layout.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "rf.h"\nint main(void) {\n'
                   '  printf("%zu", sizeof(rf_conv_desc));\n' +
                   "".join(f'  printf(" %zu", offsetof(rf_conv_desc, {"in" if n == "in_" else n}));\n' for n in names) +
                   "  return 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.run([cc, "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    want = [ctypes.sizeof(_ConvDesc)] + [getattr(_ConvDesc, n).offset for n in names]
    assert got == want


@pytest.mark.parametrize("cls,cname", [("EncoderDesc", "rf_encoder_desc"), ("EncoderLayer", "rf_encoder_layer"),
                                       ("DecoderDesc", "rf_decoder_desc"), ("DecoderLayer", "rf_decoder_layer"),
                                       ("DecoderTap", "rf_decoder_tap")])
def test_stage_desc_layout_matches_header(tmp_path, cls, cname):
    """_lib.EncoderDesc / EncoderLayer (ctypes) have the size and field offsets of rf.h's rf_encoder_desc /
    rf_encoder_layer (host C compiler on the header itself)."""
    import ctypes
    import shutil
    import subprocess
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no host C compiler")
    from renderformer_amd import _lib
    S = getattr(_lib, cls)
    names = [f[0] for f in S._fields_]
    src = tmp_path / "layout.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "rf.h"\nint main(void) {\n'
                   f'  printf("%zu", sizeof({cname}));\n' +
                   "".join(f'  printf(" %zu", offsetof({cname}, {n}));\n' for n in names) + "  return 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.run([cc, "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert got == [ctypes.sizeof(S)] + [getattr(S, n).offset for n in names]


def test_encoder_forward_validates_before_any_launch():
    """rf_encoder_forward rejects bad descriptors with RF_ERR_INVALID and a message, before touching the device
    (runs without a GPU); an empty stack is a no-op."""
    import ctypes
    from renderformer_amd import _lib
    lib = _lib.load(require_device=False)
    fwd = lambda d, x=1: int(lib.rf_encoder_forward(x, 1024, ctypes.addressof(d), None))  # noqa: E731
    assert lib.rf_encoder_forward(None, 0, None, None) == 1
    assert fwd(_lib.EncoderDesc(n_layers=0, rows=5)) == 0
    layers = (_lib.EncoderLayer * 1)()
    good = dict(n_layers=1, rows=64, dim=1024, n_heads=8, ffn_dim=4096, operand_dtype=1, eps=1e-6,
                layers=ctypes.addressof(layers), problems=1, n_problems=1, workspace=256, attn_ws=256)
    for bad, msg in ((dict(dim=1000), b"n_heads"), (dict(operand_dtype=7), b"operand_dtype"),
                     (dict(ffn_dim=100), b"ffn_dim"), (dict(workspace=0), b"null pointer"),
                     (dict(pos=16), b"freqs"), (dict(n_problems=0), b"problems")):
        assert fwd(_lib.EncoderDesc(**{**good, **bad})) == 1, bad
        assert msg in lib.rf_last_error(), (bad, lib.rf_last_error())
    assert fwd(_lib.EncoderDesc(**good)) == 1 and b"layer 0" in lib.rf_last_error()  # null weights
    assert lib.rf_encoder_workspace_bytes(5649, 1024, 4096, 1) >= 5649 * (5 * 1024 + 4096) * 2


def test_decoder_forward_validates_before_any_launch():
    """rf_decoder_forward rejects bad descriptors with RF_ERR_INVALID and a message before touching the device;
    rf_decoder_workspace_bytes sizes the batched K/V and keys of every layer."""
    import ctypes
    from renderformer_amd import _lib
    lib = _lib.load(require_device=False)
    fwd = lambda d: int(lib.rf_decoder_forward(1, 1024, ctypes.addressof(d), None))  # noqa: E731
    assert fwd(_lib.DecoderDesc(n_layers=0, rows=5)) == 0
    layers = (_lib.DecoderLayer * 2)()
    for L in layers:
        L.query_norm = L.w_q = L.w_out = L.ffn_norm = L.w13 = L.w2 = 256
    taps = (_lib.DecoderTap * 2)()
    taps[0].layer, taps[0].p_hi, taps[0].p_ld = 1, 256, 1024
    taps[1].layer, taps[1].p_hi, taps[1].p_ld = 0, 256, 1024  # out of layer order
    good = dict(n_layers=2, rows=4096, dim=1024, n_heads=8, ffn_dim=4096, operand_dtype=1, eps=1e-6,
                layers=ctypes.addressof(layers), ctx=256, ld_ctx=1024, ctx_rows=5649, ctx_dim=1024, ctx_norm=256,
                w_kv_all=256, kv_rows=5649, kv_src_rows=256, k_batch=1, cross_problems=256, n_cross=1,
                workspace=256, attn_ws=256)
    for bad, msg in ((dict(dim=1000), b"n_heads"), (dict(ctx_dim=1000), b"ctx_dim"), (dict(n_cross=0), b"problems"),
                     (dict(w_kv_all=0, k_batch=0), b"K/V weights"), (dict(w_kv_all=0), b"k_batch"),
                     (dict(kv_pos=16), b"freqs"), (dict(ray_pos=16, freqs=16, n_freqs=6, ld_ray_pos=9), b"ray_pos"),
                     (dict(taps=ctypes.addressof(taps), n_taps=2), b"tap 1")):
        assert fwd(_lib.DecoderDesc(**{**good, **bad})) == 1, bad
        assert msg in lib.rf_last_error(), (bad, lib.rf_last_error())
    layers[1].self_norm = 256  # self-attention weights for one layer only
    assert fwd(_lib.DecoderDesc(**good)) == 1 and b"every layer or none" in lib.rf_last_error()
    d = _lib.DecoderDesc(**good)
    one = int(lib.rf_decoder_workspace_bytes(ctypes.addressof(d)))
    assert one >= 2 * (4096 * (3 * 1024 + 4096) + 5649 * 1024 * (1 + 2 * 2 + 2))  # h/q2/att, g, hc, kv_all, kview_all


def test_production_build_refuses_study_kernels():
    """the measured-slower alternatives and ablation variants live in the study build only; the
    production librfhip refuses a request for one with RF_ERR_UNSUPPORTED (before any launch, so no device is
    needed) instead of running something else or garbage."""
    import ctypes

    import torch  # noqa: F401
    from renderformer_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("librfhip.so not built")
    lib = _lib.load(require_device=False)
    if _lib.study_build():
        pytest.skip("RF_LIB points at the study build")
    # the legacy split-KV path (n_split >= 1) and its merge
    rc = lib.rf_attn_fwd(ctypes.c_void_p(16), 256, ctypes.c_void_p(16), 256, ctypes.c_void_p(16), 256,
                         ctypes.c_void_p(16), 256, ctypes.c_void_p(16), 1, 10, 2, 128, 1.0, 2, ctypes.c_void_p(16),
                         10, None)
    assert rc == 3 and b"study" in lib.rf_last_error()
    rc = lib.rf_attn_combine(ctypes.c_void_p(16), 10, 2, 2, None, 10, ctypes.c_void_p(16), 256, None)
    assert rc == 3 and b"study" in lib.rf_last_error()
