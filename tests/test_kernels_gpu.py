"""Per-kernel numerics of librfhip against fp32/fp64 PyTorch references of the same op.

Inputs are rounded to bf16 first, so the reference sees exactly the kernel's
operands; remaining differences are accumulation order and output rounding.
"""
import math

import pytest
import torch
import torch.nn.functional as F
from conftest import needs_study

from oracle import rf_ref

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from renderformer_amd import _lib
    _lib.load()


def _ops():
    from renderformer_amd import ops
    return ops


def relerr(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("m,n,k", [(1, 128, 64), (77, 256, 128), (333, 384, 192), (5649, 1024, 1024),
                                   (1000, 128, 13312), (4096, 3072, 1024), (5649, 1024, 4096), (4096, 1024, 4096),
                                   (5649, 3072, 1024), (5649, 20480, 1024)])
def test_gemm_f32_bf16(m, n, k):
    """Plain epilogues (bf16 out, fp32 + bias, fp32 residual accumulate) on the hand-written engine with the
    tile the cost model picks for the shape (the path's projection shapes included), against fp64."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(m * 7 + n)
    a = torch.randn(m, k, generator=g).bfloat16().to(dev)
    w = (torch.randn(n, k, generator=g) / math.sqrt(k)).bfloat16().to(dev)
    bias = torch.randn(n, generator=g).to(dev)
    ref = a.double() @ w.double().t() + bias.double()
    out = torch.empty(m, n, device=dev)
    ops.gemm(a, w, out, bias, ops.EPI_F32)
    assert relerr(out, ref) < 1e-5
    outb = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    ops.gemm(a, w, outb, bias, ops.EPI_BF16)
    assert relerr(outb.float(), ref) < 4e-3
    acc = torch.randn(m, n, generator=g).to(dev)
    ref2 = acc.double() + ref
    ops.gemm(a, w, acc, bias, ops.EPI_ADD_F32)
    assert relerr(acc, ref2) < 1e-5


@pytest.mark.parametrize("grid", ["512", "768", "37", "sk256", "skph"])
@pytest.mark.parametrize("m,n,k", [(1000, 1024, 1024), (300, 256, 4096), (129, 128, 96), (5649, 1024, 64),
                                   (5649, 1024, 4096), (4096, 3072, 1024)])
def test_gemm_stream_k(monkeypatch, grid, m, n, k):
    """Stream-K split (forced grid sizes, incl. an odd one where a tile spans 3+ blocks, and the 256x256-tile
    variant over 256 blocks) vs fp64, every epilogue (engine backend)."""
    ops = _ops()
    if grid in ("sk256", "skph"):
        if n % 256 or (grid == "skph" and k % 64):
            pytest.skip("256x256 tiles need N % 256 == 0 (and K % 64 == 0 for the phased loop)")
        monkeypatch.setenv("RF_GEMM_SK256" if grid == "sk256" else "RF_GEMM_SKPH", "1")
        monkeypatch.setenv("RF_GEMM_PHASED", "0" if grid == "sk256" else "1")
    else:
        monkeypatch.setenv("RF_GEMM_SK", grid)
    g = torch.Generator(device="cpu").manual_seed(m + n + k)
    a = torch.randn(m, k, generator=g).bfloat16().to(dev)
    w = (torch.randn(n, k, generator=g) / math.sqrt(k)).bfloat16().to(dev)
    bias = torch.randn(n, generator=g).to(dev)
    ref = a.double() @ w.double().t() + bias.double()
    for _ in range(2):  # second pass reuses the workspace flags with a new epoch
        out = torch.empty(m, n, device=dev)
        ops.gemm(a, w, out, bias, ops.EPI_F32)
        assert relerr(out, ref) < 1e-5
    acc = torch.randn(m, n, generator=g).to(dev)
    ref2 = acc.double() + ref
    ops.gemm(a, w, acc, bias, ops.EPI_ADD_F32)
    assert relerr(acc, ref2) < 1e-5
    outb = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    ops.gemm(a, w, outb, bias, ops.EPI_BF16)
    assert relerr(outb.float(), ref) < 4e-3
    from renderformer_amd.model import _interleave_swiglu
    outs = torch.empty(m, n // 2, device=dev, dtype=torch.bfloat16)
    ops.gemm(a, _interleave_swiglu(w[: n // 2].cpu(), w[n // 2:].cpu()).to(dev), outs, None, ops.EPI_SWIGLU)
    refs = F.silu(a.double() @ w[: n // 2].double().t()) * (a.double() @ w[n // 2:].double().t())
    assert relerr(outs.float(), refs) < 5e-3


TILES = {"256ph": "256", "128x256ph": "1282", "96x256ph": "963", "64x256ph": "643", "256ring": "256",
         "96x256ring": "962", "64x256ring": "642", "64x256ring4w": "644", "128ring": "128",
         "128x256ph3": "1283", "96x256ph3": "964", "64x256ph3": "645", "128ring8wk64": "12884", "128ringk64": "12823",
         "96x256ringk64": "9623", "96x256ring6": "966"}


@pytest.mark.parametrize("tile", list(TILES))
@pytest.mark.parametrize("m,n,k", [(1, 256, 64), (300, 512, 128), (777, 256, 192), (5649, 3072, 1024),
                                   (4096, 1024, 4096), (2000, 768, 320), (5649, 1024, 1024)])
def test_gemm_256_tiles(monkeypatch, tile, m, n, k):
    """Every tile shape of the engine (phased BK=64 loop at 256/128/96/64 x 256 — the short ones stage A from
    only some waves —, the ring engine's 256x256, 96x256, 64x256 and 128x128), forced on every shape (ragged M,
    one to three K-tiles, long K), every epilogue (the residual one starting from the C tile), vs fp64."""
    ops = _ops()
    monkeypatch.setenv("RF_GEMM_TILE", TILES[tile])
    monkeypatch.setenv("RF_GEMM_PHASED", "0" if tile == "256ring" else "1")
    g = torch.Generator(device="cpu").manual_seed(m + 3 * n + k)
    a = torch.randn(m, k, generator=g).bfloat16().to(dev)
    w = (torch.randn(n, k, generator=g) / math.sqrt(k)).bfloat16().to(dev)
    bias = torch.randn(n, generator=g).to(dev)
    ref = a.double() @ w.double().t() + bias.double()
    out = torch.empty(m, n, device=dev)
    ops.gemm(a, w, out, bias, ops.EPI_F32)
    assert relerr(out, ref) < 1e-5
    acc = torch.randn(m, n, generator=g).to(dev)
    ref2 = acc.double() + ref
    ops.gemm(a, w, acc, bias, ops.EPI_ADD_F32)
    assert relerr(acc, ref2) < 1e-5
    outb = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    ops.gemm(a, w, outb, bias, ops.EPI_BF16)
    assert relerr(outb.float(), ref) < 4e-3
    from renderformer_amd.model import _interleave_swiglu
    outs = torch.empty(m, n // 2, device=dev, dtype=torch.bfloat16)
    ops.gemm(a, _interleave_swiglu(w[: n // 2].cpu(), w[n // 2:].cpu()).to(dev), outs, None, ops.EPI_SWIGLU)
    refs = F.silu(a.double() @ w[: n // 2].double().t()) * (a.double() @ w[n // 2:].double().t())
    assert relerr(outs.float(), refs) < 5e-3


F16_TILES = {"auto": None, "256ph": "256", "128x256ph": "1282", "96x256ph3": "964", "64x256ph3": "645",
             "128x256ph3": "1283", "96x256ring": "962", "128ring8wk64": "12884", "128ring": "128", "skph": "skph",
             "quad": "quad1", "quadsk": "quad2", "quad128x192": "quad1@128x192", "quad160x256sk": "quad2@160x256",
             "quad128x128": "quad1@128x128"}


@pytest.mark.parametrize("tile", list(F16_TILES))
@pytest.mark.parametrize("m,n,k", [(1, 256, 64), (777, 256, 192), (5649, 3072, 1024), (4096, 1024, 4096),
                                   (5649, 1024, 1024), (4096, 8192, 1024), (300, 512, 256), (1000, 768, 384)])
def test_gemm_f16_operands(monkeypatch, tile, m, n, k):
    """rf_gemm_f16 (fp16 A and W, fp16 MFMAs) on every loop the cost model can pick, every epilogue incl. the
    fp16 outputs (RF_EPI_F16, RF_EPI_SWIGLU_F16) and the bf16 one, vs fp64 of the same fp16 operands."""
    ops = _ops()
    if F16_TILES[tile] == "skph":
        if (m + 255) // 256 * (n // 256) < 512:
            pytest.skip("the phased stream-K path needs >= 512 whole 256x256 tiles")
        monkeypatch.setenv("RF_GEMM_SKPH", "1")
    elif (F16_TILES[tile] or "").startswith("quad"):
        needs_study("the 4-wave GEMM")
        mode, _, qt = F16_TILES[tile][4:].partition("@")
        bn = int(qt.split("x")[1]) if qt else 256
        if k % 128 or n % bn:
            pytest.skip("the 4-wave engine needs K % 128 == 0 (and whole column tiles for the SwiGLU check)")
        monkeypatch.setenv("RF_GEMM_QUAD", mode)
        if qt:
            monkeypatch.setenv("RF_GEMM_QUAD_TILE", qt)
    elif F16_TILES[tile]:
        monkeypatch.setenv("RF_GEMM_TILE", F16_TILES[tile])
    g = torch.Generator(device="cpu").manual_seed(m + 5 * n + k)
    a = torch.randn(m, k, generator=g).half().to(dev)
    w = (torch.randn(n, k, generator=g) / math.sqrt(k)).half().to(dev)
    bias = torch.randn(n, generator=g).to(dev)
    ref = a.double() @ w.double().t() + bias.double()
    out = torch.empty(m, n, device=dev)
    ops.gemm(a, w, out, bias, ops.EPI_F32)
    assert relerr(out, ref) < 1e-5
    acc = torch.randn(m, n, generator=g).to(dev)
    ref2 = acc.double() + ref
    ops.gemm(a, w, acc, bias, ops.EPI_ADD_F32)
    assert relerr(acc, ref2) < 1e-5
    for dt, tol in ((torch.float16, 6e-4), (torch.bfloat16, 4e-3)):
        o16 = torch.empty(m, n, device=dev, dtype=dt)
        ops.gemm(a, w, o16, bias, ops.EPI_BF16)
        assert relerr(o16.float(), ref) < tol, dt
    from renderformer_amd.model import _interleave_swiglu
    refs = F.silu(a.double() @ w[: n // 2].double().t()) * (a.double() @ w[n // 2:].double().t())
    for dt, tol in ((torch.float16, 8e-4), (torch.bfloat16, 5e-3)):
        outs = torch.empty(m, n // 2, device=dev, dtype=dt)
        ops.gemm(a, _interleave_swiglu(w[: n // 2].cpu(), w[n // 2:].cpu()).to(dev), outs, None, ops.EPI_SWIGLU)
        assert relerr(outs.float(), refs) < tol, dt


@pytest.mark.parametrize("tile", ["256x256", "128x192", "160x256"])
@pytest.mark.parametrize("stg", ["1", "0"])
@pytest.mark.parametrize("mode", ["1", "2"])
@pytest.mark.parametrize("m,n,k", [(5649, 8192, 1024), (513, 2048, 640), (8192, 512, 2048), (777, 1024, 384)])
def test_gemm_quad_bf16_and_persistent(monkeypatch, tile, mode, stg, m, n, k):
    """The 4-wave engine (RF_GEMM_QUAD: 1 data-parallel / persistent over whole tiles, 2 stream-K over pairs of
    K-tiles; register or LDS-DMA staging; 256x256 / 128x192 / 160x256 tiles) on bf16 operands: more tiles than CUs
    (persistent), ragged rows and ragged column tiles, odd K-pair counts split over blocks; fp32, residual and
    SwiGLU epilogues vs fp64 (SwiGLU with a ragged column tile runs on the default engine)."""
    needs_study("the 4-wave GEMM")
    monkeypatch.setenv("RF_GEMM_QUAD", mode)
    monkeypatch.setenv("RF_GEMM_QUAD_STG", stg)  # register staging (default) / LDS-DMA
    monkeypatch.setenv("RF_GEMM_QUAD_TILE", tile)  # 128x192: a ragged last column tile when 192 does not divide N
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(m + n + k)
    a = torch.randn(m, k, generator=g).bfloat16().to(dev)
    w = (torch.randn(n, k, generator=g) / math.sqrt(k)).bfloat16().to(dev)
    ref = a.double() @ w.double().t()
    out = torch.empty(m, n, device=dev)
    ops.gemm(a, w, out, None, ops.EPI_F32)
    assert relerr(out, ref) < 1e-5
    acc = torch.randn(m, n, generator=g).to(dev)
    ref2 = acc.double() + ref
    ops.gemm(a, w, acc, None, ops.EPI_ADD_F32)
    assert relerr(acc, ref2) < 1e-5
    from renderformer_amd.model import _interleave_swiglu
    outs = torch.empty(m, n // 2, device=dev, dtype=torch.bfloat16)
    ops.gemm(a, _interleave_swiglu(w[: n // 2].cpu(), w[n // 2:].cpu()).to(dev), outs, None, ops.EPI_SWIGLU)
    refs = F.silu(a.double() @ w[: n // 2].double().t()) * (a.double() @ w[n // 2:].double().t())
    assert relerr(outs.float(), refs) < 5e-3
    assert ops.load().rf_device_error() == 0


def test_rmsnorm_f16_and_attention_f16_out():
    """The fp16-output forms feeding fp16 GEMMs: rf_rmsnorm_f16, and the stream-K / Swin attention writing O as
    fp16 (q/k/v bf16): the same values as the bf16-output launches up to the output rounding."""
    ops = _ops()
    x = torch.randn(333, 1024, device=dev) * 3
    w = torch.rand(1024, device=dev) + 0.5
    ref = F.rms_norm(x.double(), (1024,), w.double(), 1e-6)
    out = torch.empty(333, 1024, device=dev, dtype=torch.float16)
    ops.rmsnorm(x, w, 1e-6, out)
    assert relerr(out.float(), ref) < 6e-4
    H, D = 8, 1024
    g = torch.Generator(device="cpu").manual_seed(5)
    lens = [700, 129, 65]
    T = sum(lens)
    qkv = torch.randn(T, 3 * D, generator=g).bfloat16().to(dev)
    probs, off = [], 0
    for n in lens:
        probs.append([off, n, off, n, off])
        off += n
    pt = torch.tensor(probs, dtype=torch.int32, device=dev)
    outs = {}
    for dt in (torch.bfloat16, torch.float16):
        o = torch.zeros(T, D, device=dev, dtype=dt)
        ops.attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], o, pt, max(lens), H,
                      schedule=ops.attn_schedule(probs, H, dev))
        outs[dt] = o.float()
    off = 0
    for n in lens:
        sl = slice(off, off + n)
        r = _ref_attn(qkv[sl, :D].float().cpu(), qkv[sl, D:2 * D].float().cpu(), qkv[sl, 2 * D:].float().cpu(), H)
        assert relerr(outs[torch.float16][sl].cpu(), r) < 2e-3
        assert relerr(outs[torch.bfloat16][sl].cpu(), r) < 6e-3
        off += n
    n_img, gh = 2, 16
    T2 = n_img * gh * gh
    qkv2 = torch.randn(T2, 3 * D, generator=g).bfloat16().to(dev)
    sw = {}
    for dt in (torch.bfloat16, torch.float16):
        o = torch.zeros(T2, D, device=dev, dtype=dt)
        ops.swin_attention(qkv2[:, :D], qkv2[:, D:2 * D], qkv2[:, 2 * D:], o, n_img, gh, gh, 4, H)
        sw[dt] = o.float()
    assert relerr(sw[torch.float16], sw[torch.bfloat16]) < 4e-3


def test_f16_range_flag_writers():
    """Every fp16 writer raises the range flag on a value beyond fp16's range (|x| > 65504, inf included) and
    only then: the fp16 GEMM epilogues (plain and SwiGLU), rf_rmsnorm_f16, the attention / Swin fp16 O and the
    fp16 plane of rf_split_planes; bf16 outputs of the same values never raise it."""
    from renderformer_amd import ops
    ops.clear_f16_range_flag()
    g = torch.Generator(device="cpu").manual_seed(99)
    a = torch.randn(300, 256, generator=g).half().to(dev)
    w = (torch.randn(512, 256, generator=g) / 16).half().to(dev)

    def flag_after(fn):
        ops.clear_f16_range_flag()
        fn()
        torch.cuda.synchronize()
        f = ops.f16_range_flag()
        ops.clear_f16_range_flag()
        return f

    o16 = torch.empty(300, 512, device=dev, dtype=torch.float16)
    assert flag_after(lambda: ops.gemm(a, w, o16)) == 0
    assert flag_after(lambda: ops.gemm(a * 16, w * 4096, o16)) != 0               # |x| ~ 6.6e4 (1 sigma)
    assert flag_after(lambda: ops.gemm(a * 16, w * 4096, torch.empty_like(o16, dtype=torch.bfloat16))) == 0
    sw = torch.empty(300, 256, device=dev, dtype=torch.float16)
    assert flag_after(lambda: ops.gemm(a, w, sw, None, ops.EPI_SWIGLU)) == 0
    assert flag_after(lambda: ops.gemm(a, w * 2000, sw, None, ops.EPI_SWIGLU)) != 0  # silu(g) u ~ 4e6
    x = torch.randn(64, 1024, generator=g).to(dev)
    h = torch.empty(64, 1024, device=dev, dtype=torch.float16)
    assert flag_after(lambda: ops.rmsnorm(x, torch.ones(1024, device=dev), 1e-6, h)) == 0
    assert flag_after(lambda: ops.rmsnorm(x, torch.full((1024,), 1e5, device=dev), 1e-6, h)) != 0
    H, D, S = 2, 256, 200
    q = torch.randn(S, D, generator=g).bfloat16().to(dev)
    k = torch.randn(S, D, generator=g).bfloat16().to(dev)
    v = torch.randn(S, D, generator=g).bfloat16().to(dev)
    pt = torch.tensor([[0, S, 0, S, 0]], dtype=torch.int32, device=dev)
    oa = torch.empty(S, D, device=dev, dtype=torch.float16)
    assert flag_after(lambda: ops.attention(q, k, v, oa, pt, S, H)) == 0
    assert flag_after(lambda: ops.attention(q, k, (v.float() * 1e7).bfloat16(), oa, pt, S, H)) != 0
    assert flag_after(lambda: ops.attention(q, k, (v.float() * 1e7).bfloat16(), oa.bfloat16(), pt, S, H)) == 0
    n_img, gs = 1, 8
    qs = torch.randn(n_img * gs * gs, D, generator=g).bfloat16().to(dev)
    os_ = torch.empty(n_img * gs * gs, D, device=dev, dtype=torch.float16)
    assert flag_after(lambda: ops.swin_attention(qs, qs, qs, os_, n_img, gs, gs, 0, H)) == 0
    assert flag_after(lambda: ops.swin_attention(qs, qs, (qs.float() * 1e7).bfloat16(), os_, n_img, gs, gs, 0, H)) != 0
    from renderformer_amd import _lib
    xs = torch.randn(128, 64, generator=g).to(dev)
    plane = torch.empty(128, 64, device=dev, dtype=torch.float16)
    split = lambda t: _lib.call("rf_split_planes", t.data_ptr(), 128, 64, 64, plane.data_ptr(), None, 64, 0,  # noqa: E731
                                _lib.stream())
    assert flag_after(lambda: split(xs)) == 0
    assert flag_after(lambda: split(xs * 1e6)) != 0


def test_range_words_are_per_render():
    """rf_range_word_* (ABI 14): a bound word collects exactly the overflows of the launches issued while it is
    bound on this thread; another word and the process-wide word stay clear; unbinding returns to the process
    word; a word bound on another thread does not capture this thread's launches."""
    import ctypes
    import threading
    from renderformer_amd import _lib, ops
    lib = _lib.load()
    ops.clear_f16_range_flag()
    words = []
    for _ in range(2):
        h = ctypes.c_void_p()
        assert lib.rf_range_word_new(ctypes.byref(h)) == 0 and h.value
        words.append(h.value)
    wa, wb = words
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(64, 1024, generator=g).to(dev)
    h16 = torch.empty(64, 1024, device=dev, dtype=torch.float16)
    big = torch.full((1024,), 1e5, device=dev)
    lib.rf_range_word_bind(wa)
    ops.rmsnorm(x, big, 1e-6, h16)                               # overflows: raises word A
    lib.rf_range_word_bind(wb)
    ops.rmsnorm(x, torch.ones(1024, device=dev), 1e-6, h16)      # in range: word B stays 0
    seen = {}

    def other_thread():  # this thread's binding is B; a launch from a thread with nothing bound -> process word
        ops.rmsnorm(x, big, 1e-6, h16)
        torch.cuda.synchronize()
        seen["global"] = ops.f16_range_flag()
    t = threading.Thread(target=other_thread)
    t.start()
    t.join()
    lib.rf_range_word_bind(None)
    torch.cuda.synchronize()
    assert lib.rf_range_word_read(wa) == 2 and lib.rf_range_word_read(wb) == 0
    assert seen["global"] == 2
    ops.clear_f16_range_flag()
    ops.rmsnorm(x, big, 1e-6, h16)                               # unbound again: the process word
    torch.cuda.synchronize()
    assert ops.f16_range_flag() == 2 and lib.rf_range_word_read(wa) == 2
    lib.rf_range_word_clear(wa)
    assert lib.rf_range_word_read(wa) == 0
    ops.clear_f16_range_flag()
    for w in words:
        assert lib.rf_range_word_free(w) == 0


def test_gemm_asymmetric_identity():
    """A = I with an asymmetric W catches a transposed C write (guide §3)."""
    ops = _ops()
    n = 128
    a = torch.eye(n, 128, device=dev).bfloat16()
    w = (torch.arange(n * 128, device=dev).float().view(n, 128) % 251).bfloat16()
    out = torch.empty(n, n, device=dev)
    ops.gemm(a, w, out, None, ops.EPI_F32)
    assert torch.equal(out, w.float().t())


@pytest.mark.parametrize("m,f,k", [(77, 512, 256), (1234, 3072, 768)])
def test_gemm_swiglu(m, f, k):
    ops = _ops()
    from renderformer_amd.model import _interleave_swiglu
    g = torch.Generator(device="cpu").manual_seed(f)
    a = torch.randn(m, k, generator=g).bfloat16()
    w1 = (torch.randn(f, k, generator=g) / math.sqrt(k)).bfloat16()
    w3 = (torch.randn(f, k, generator=g) / math.sqrt(k)).bfloat16()
    ref = F.silu(a.double() @ w1.double().t()) * (a.double() @ w3.double().t())
    out = torch.empty(m, f, device=dev, dtype=torch.bfloat16)
    ops.gemm(a.to(dev), _interleave_swiglu(w1, w3).to(dev), out, None, ops.EPI_SWIGLU)
    assert relerr(out.float().cpu(), ref) < 5e-3


def test_rmsnorm():
    ops = _ops()
    x = torch.randn(333, 768, device=dev) * 3
    w = torch.rand(768, device=dev) + 0.5
    out = torch.empty(333, 768, device=dev, dtype=torch.bfloat16)
    ops.rmsnorm(x, w, 1e-6, out)
    ref = F.rms_norm(x.double(), (768,), w.double(), 1e-6)
    assert relerr(out.float(), ref) < 4e-3


def test_qk_norm_rope_matches_oracle():
    ops = _ops()
    T, H = 300, 8
    D = H * 128
    src = torch.randn(T, 3 * D).bfloat16()
    w = torch.rand(D) + 0.5
    pos = torch.rand(T, 9) * 2 - 1
    freqs = 2 ** torch.linspace(0, math.log2(5), 6)
    q = src[:, :D].float()
    qn = F.rms_norm(q, (D,), w, 1e-6)
    cos, sin = rf_ref.rope_cos_sin(pos[None], freqs, 128)
    ref = rf_ref.rope_apply(qn.view(1, T, H, 128).transpose(1, 2), cos, sin).transpose(1, 2).reshape(T, D)
    s = src.to(dev)
    ops.qk_norm_rope(s[:, :D], s[:, :D], H, w.to(dev), 1e-6, pos.to(dev), freqs.to(dev))
    assert relerr(s[:, :D].float().cpu(), ref) < 4e-3
    assert torch.equal(s[:, D:].cpu(), src[:, D:])  # other columns untouched
    # gather + per-row pos divisor (ray tokens: one position per view)
    rows = torch.tensor([5, 0, 299, 5], dtype=torch.int32)
    dst = torch.empty(4, D, device=dev, dtype=torch.bfloat16)
    vpos = torch.rand(2, 9)
    ops.qk_norm_rope(src[:, D:2 * D].to(dev), dst, H, None, 1e-6, vpos.to(dev), freqs.to(dev), pos_div=2,
                     src_rows=rows.to(dev))
    kk = src[:, D:2 * D].float()[rows.long()]
    cos, sin = rf_ref.rope_cos_sin(vpos.repeat_interleave(2, 0)[None], freqs, 128)
    ref2 = rf_ref.rope_apply(kk.view(1, 4, H, 128).transpose(1, 2), cos, sin).transpose(1, 2).reshape(4, D)
    assert relerr(dst.float().cpu(), ref2) < 4e-3


def test_qk_norm_rope_two_segments():
    """q and k of one qkv row in a single launch, each with its own full-width norm."""
    ops = _ops()
    T, H = 77, 2
    D = H * 128
    src = torch.randn(T, 3 * D).bfloat16()
    w = torch.rand(2 * D) + 0.5
    pos = torch.rand(T, 9) * 2 - 1
    freqs = 2 ** torch.linspace(0, math.log2(5), 6)
    cos, sin = rf_ref.rope_cos_sin(pos[None], freqs, 128)
    s = src.to(dev)
    ops.qk_norm_rope(s[:, :2 * D], s[:, :2 * D], H, w.to(dev), 1e-6, pos.to(dev), freqs.to(dev), n_seg=2)
    for sg in range(2):
        x = F.rms_norm(src[:, sg * D:(sg + 1) * D].float(), (D,), w[sg * D:(sg + 1) * D], 1e-6)
        ref = rf_ref.rope_apply(x.view(1, T, H, 128).transpose(1, 2), cos, sin).transpose(1, 2).reshape(T, D)
        assert relerr(s[:, sg * D:(sg + 1) * D].float().cpu(), ref) < 4e-3
    assert torch.equal(s[:, 2 * D:].cpu(), src[:, 2 * D:])


@pytest.mark.parametrize("rows,H", [(5649, 8), (77, 2)])
def test_qk_norm_rope_split_segments_bit_identical(monkeypatch, rows, H):
    """The q/k pair run as two one-segment groups (default) equals the two-segment wave (RF_QKN_SPLIT=0) bit for bit,
    q scale on q only."""
    ops = _ops()
    D = H * 128
    g = torch.Generator(device="cpu").manual_seed(rows)
    src = torch.randn(rows, 3 * D, generator=g).bfloat16().to(dev)
    w = (torch.rand(2 * D, generator=g) + 0.5).to(dev)
    pos = (torch.rand(rows, 9, generator=g) * 2 - 1).to(dev)
    freqs = (2 ** torch.linspace(0, math.log2(5), 6)).to(dev)
    outs = []
    for split in ("1", "0"):
        monkeypatch.setenv("RF_QKN_SPLIT", split)
        s = src.clone()
        ops.qk_norm_rope(s[:, :2 * D], s[:, :2 * D], H, w, 1e-6, pos, freqs, n_seg=2, q_scale=ops.Q_LOG2_SCALE)
        outs.append(s)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("with_norm", [True, False])
def test_qk_norm_rope_groups_equals_per_group(with_norm):
    """One launch over the keys of every decoder layer (the K columns at stride 2D of the batched K/V
    projection, gathered per view) is bit-identical to one launch per layer, and matches the oracle."""
    ops = _ops()
    T, H, G = 131, 8, 3
    D = H * 128
    kv = torch.randn(T, G * 2 * D).bfloat16().to(dev)
    w = (torch.rand(G * D) + 0.5).to(dev) if with_norm else None
    rows = torch.tensor(list(range(T)) + list(range(0, T, 2)), dtype=torch.int32)  # two views of one scene
    pos = (torch.rand(rows.numel(), 9) * 2 - 1).to(dev)
    freqs = (2 ** torch.linspace(0, math.log2(5), 6)).to(dev)
    out = torch.empty(rows.numel(), G * D, device=dev, dtype=torch.bfloat16)
    ops.qk_norm_rope_groups(kv, 2 * D, out, D, G, H, w, 1e-6, pos, freqs, src_rows=rows.to(dev))
    cos, sin = rf_ref.rope_cos_sin(pos.cpu()[None], freqs.cpu(), 128)
    for g in range(G):
        one = torch.empty(rows.numel(), D, device=dev, dtype=torch.bfloat16)
        wg = w[g * D:(g + 1) * D] if with_norm else None
        ops.qk_norm_rope(kv[:, 2 * D * g:2 * D * g + D], one, H, wg, 1e-6, pos, freqs, src_rows=rows.to(dev))
        assert torch.equal(out[:, g * D:(g + 1) * D], one)
        x = kv[:, 2 * D * g:2 * D * g + D].float().cpu()[rows.long()]
        if with_norm:
            x = F.rms_norm(x, (D,), wg.cpu(), 1e-6)
        ref = rf_ref.rope_apply(x.view(1, -1, H, 128).transpose(1, 2), cos, sin).transpose(1, 2).reshape(-1, D)
        assert relerr(out[:, g * D:(g + 1) * D].float().cpu(), ref) < 4e-3


def test_qk_norm_rope_groups_scale_applies_to_every_group():
    """rf_qk_norm_rope_groups with seg0_scale != 1 scales segment 0 of EVERY group (rf.h: the
    function is rf_qk_norm_rope applied per group); only the host's internal q/k split of one two-segment group
    scales group 0 alone.  Bit-identical to one rf_qk_norm_rope launch per group with the same q_scale."""
    ops = _ops()
    T, H, G = 97, 8, 3
    D = H * 128
    kv = torch.randn(T, G * 2 * D).bfloat16().to(dev)
    w = (torch.rand(G * D) + 0.5).to(dev)
    pos = (torch.rand(T, 9) * 2 - 1).to(dev)
    freqs = (2 ** torch.linspace(0, math.log2(5), 6)).to(dev)
    out = torch.empty(T, G * D, device=dev, dtype=torch.bfloat16)
    ops.qk_norm_rope_groups(kv, 2 * D, out, D, G, H, w, 1e-6, pos, freqs, seg0_scale=2.5)
    for g in range(G):
        one = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
        ops.qk_norm_rope(kv[:, 2 * D * g:2 * D * g + D], one, H, w[g * D:(g + 1) * D], 1e-6, pos, freqs, q_scale=2.5)
        assert torch.equal(out[:, g * D:(g + 1) * D], one), g


def _ref_attn(q, k, v, H):
    lq, lk = q.shape[0], k.shape[0]
    qh = q.double().view(lq, H, 128).transpose(0, 1)
    kh = k.double().view(lk, H, 128).transpose(0, 1)
    vh = v.double().view(lk, H, 128).transpose(0, 1)
    s = qh @ kh.transpose(1, 2) / math.sqrt(128)
    return (torch.softmax(s, -1) @ vh).transpose(0, 1).reshape(lq, H * 128)


@pytest.fixture(params=["sk", "sk_grid7", "sk_grid61", "p4", "p4_grid7", "p4_grid61", "legacy"])
def attn_mode(request, monkeypatch):
    """Varlen attention modes: the stream-K kernel on the full grid, on small grids that cut most units
    into 2-3 pieces merged by their owner (RF_ATTN_GRID), the same for the one-wave-per-SIMD stream-K kernel
    (RF_ATTN_P4=1), and the legacy per-unit kernel (n_split=1).  Returns the n_split to pass."""
    if request.param.startswith("p4") or request.param == "legacy":
        needs_study("the one-wave-per-SIMD / legacy split-KV attention")
    if request.param.startswith("p4"):
        monkeypatch.setenv("RF_ATTN_P4", "1")
    if "_grid" in request.param:
        monkeypatch.setenv("RF_ATTN_GRID", request.param.split("_grid")[1])
    return 1 if request.param == "legacy" else None


@pytest.fixture(params=["sk", "p4"])
def sk_kernel(request, monkeypatch):
    """The two stream-K kernels: 8 waves x 32 rows (default) and 4 waves x 64 rows (RF_ATTN_P4=1)."""
    if request.param == "p4":
        needs_study("the one-wave-per-SIMD attention")
    monkeypatch.setenv("RF_ATTN_P4", "1" if request.param == "p4" else "0")
    return request.param


@pytest.mark.parametrize("lens", [[1], [63], [64, 65], [77, 200, 1], [5649]])
def test_attention_varlen_self(lens, attn_mode):
    ops = _ops()
    H = 2
    D = H * 128
    T = sum(lens)
    g = torch.Generator(device="cpu").manual_seed(sum(lens))
    qkv = (torch.randn(T, 3 * D, generator=g) * 2).bfloat16()
    probs, off = [], 0
    for n in lens:
        probs.append([off, n, off, n, off])
        off += n
    out = torch.zeros(T, D, device=dev, dtype=torch.bfloat16)
    d = qkv.to(dev)
    ops.attention(d[:, :D], d[:, D:2 * D], d[:, 2 * D:], out, torch.tensor(probs, dtype=torch.int32, device=dev),
                  max(lens), H, n_split=attn_mode)
    out = out.float().cpu()
    off = 0
    for n in lens:
        sl = slice(off, off + n)
        ref = _ref_attn(qkv[sl, :D].float(), qkv[sl, D:2 * D].float(), qkv[sl, 2 * D:].float(), H)
        assert relerr(out[sl], ref) < 6e-3, n
        off += n


@pytest.mark.parametrize("n_split", [2, 3, 7])
def test_attention_split_kv(n_split):
    """Split-KV partials + merge: ragged problems (incl. one shorter than a key tile, so some splits see no
    keys), repeated calls on the reused workspace, and a spiked key that forces the deferred-rescale branch
    inside one split."""
    needs_study("the legacy split-KV attention")
    ops = _ops()
    H = 2
    D = H * 128
    lens = [700, 37, 300, 1]
    T = sum(lens)
    g = torch.Generator(device="cpu").manual_seed(n_split)
    qkv = torch.randn(T, 3 * D, generator=g).bfloat16()
    qkv[650, D:2 * D] = 12.0  # one large key row: its score jumps far past the running max
    probs, off = [], 0
    for n in lens:
        probs.append([off, n, off, n, off])
        off += n
    d = qkv.to(dev)
    pt = torch.tensor(probs, dtype=torch.int32, device=dev)
    for _ in range(3):
        out = torch.zeros(T, D, device=dev, dtype=torch.bfloat16)
        ops.attention(d[:, :D], d[:, D:2 * D], d[:, 2 * D:], out, pt, max(lens), H, n_split=n_split)
        o = out.float().cpu()
        off = 0
        for n in lens:
            sl = slice(off, off + n)
            ref = _ref_attn(qkv[sl, :D].float(), qkv[sl, D:2 * D].float(), qkv[sl, 2 * D:].float(), H)
            assert relerr(o[sl], ref) < 6e-3, (n_split, n)
            off += n


def test_attention_cross_shared_v(attn_mode):
    """Stage-2 form: per-view K rows, V rows shared by the views of a scene."""
    ops = _ops()
    H, D, R = 2, 256, 64
    S = [70, 33]
    Vn = 2
    g = torch.Generator(device="cpu").manual_seed(3)
    q = torch.randn(len(S) * Vn * R, D, generator=g).bfloat16()
    kview = torch.randn(sum(S) * Vn, D, generator=g).bfloat16()
    vsc = torch.randn(sum(S), D, generator=g).bfloat16()
    probs, koff, voff, p = [], 0, 0, 0
    for b, s in enumerate(S):
        for _ in range(Vn):
            probs.append([p * R, R, koff, s, voff])
            koff += s
            p += 1
        voff += s
    out = torch.empty_like(q).to(dev)
    ops.attention(q.to(dev), kview.to(dev), vsc.to(dev), out, torch.tensor(probs, dtype=torch.int32, device=dev), R, H,
                  n_split=attn_mode)
    out = out.float().cpu()
    for pr in probs:
        qs, ql, ks, kl, vs = pr
        ref = _ref_attn(q[qs:qs + ql].float(), kview[ks:ks + kl].float(), vsc[vs:vs + kl].float(), H)
        assert relerr(out[qs:qs + ql], ref) < 6e-3


@pytest.mark.parametrize("sched", [False, True])
@pytest.mark.parametrize("thr", ["8", "0"])
@pytest.mark.parametrize("grid", [None, "5", "23"])
def test_attention_stream_k_prescaled_rescale(thr, grid, sched, sk_kernel, monkeypatch):
    """The model's form: q pre-scaled by scale*log2(e) (scores are exp2 exponents, no per-score multiply),
    ragged problems with tail tiles, key spikes that force the deferred-rescale branch at chosen tiles
    (incl. right after a piece boundary), repeated launches on the re-armed workspace.  THR=0 (rescale on
    every growth) and the shipped THR=8 must both match the fp64 reference (guide rule 26).  For the p4 kernel
    the same spikes force piece replays (its running max is fixed per piece; THR=0: a replay on every growth)."""
    monkeypatch.setenv("RF_ATTN_THR", thr)
    if grid:
        monkeypatch.setenv("RF_ATTN_GRID", grid)
    ops = _ops()
    H = 4
    D = H * 128
    lens = [1000, 129, 700, 65]
    T = sum(lens)
    g = torch.Generator(device="cpu").manual_seed(7)
    qkv = torch.randn(T, 3 * D, generator=g).bfloat16()
    for r in (5, 640, 960, 1129 + 64, 1129 + 699):  # late large keys: scores jump by >> 2^8 mid-sequence
        qkv[r, D:2 * D] = (qkv[r, D:2 * D].float() * 6.0).bfloat16()
    probs, off = [], 0
    for n in lens:
        probs.append([off, n, off, n, off])
        off += n
    d = qkv.to(dev)
    qs = (d[:, :D].float() * ops.Q_LOG2_SCALE).bfloat16()
    pt = torch.tensor(probs, dtype=torch.int32, device=dev)
    # sched: the cost-balanced ranges of rf_attn_schedule (over RF_ATTN_GRID workgroups when it is set)
    sch = ops.attn_schedule(probs, H, dev) if sched else None
    for _ in range(3):
        out = torch.zeros(T, D, device=dev, dtype=torch.bfloat16)
        ops.attention(qs, d[:, D:2 * D], d[:, 2 * D:], out, pt, max(lens), H, q_prescaled=True, schedule=sch)
        o = out.float().cpu()
        off = 0
        for n in lens:
            sl = slice(off, off + n)
            qref = qs[sl].float().cpu() / ops.Q_LOG2_SCALE
            ref = _ref_attn(qref, qkv[sl, D:2 * D].float(), qkv[sl, 2 * D:].float(), H)
            assert relerr(o[sl], ref) < 6e-3, (thr, grid, n)
            off += n


@pytest.mark.parametrize("prescaled", [False, True])
@pytest.mark.parametrize("thr", ["12", "0"])
@pytest.mark.parametrize("grid", [None, "5", "23"])
def test_attention_f16_operands(grid, thr, prescaled, monkeypatch):
    """rf_attn_fwd_dt with fp16 q/k/v (the operands the reference's default torch_dtype=float16 hands
    flash_attn_varlen_*): ragged problems with tail tiles, key spikes that force the deferred rescale (THR=0: at
    every growth), cut units merged by their owners (small grids), fp16 and bf16 O; checked against fp64 at a
    tighter bar than bf16 (fp16 operands and P keep 3 more mantissa bits), and fp16 beats bf16 on the same data."""
    monkeypatch.setenv("RF_ATTN_THR", thr)
    if grid:
        monkeypatch.setenv("RF_ATTN_GRID", grid)
    ops = _ops()
    H = 4
    D = H * 128
    lens = [1000, 129, 700, 65]
    T = sum(lens)
    g = torch.Generator(device="cpu").manual_seed(17)
    qkv = torch.randn(T, 3 * D, generator=g)
    for r in (5, 640, 960, 1129 + 64, 1129 + 699):
        qkv[r, D:2 * D] *= 6.0
    qkv[:, 2 * D:] *= 1000.0  # values far outside bf16's 8-bit mantissa comfort, well inside fp16's range
    probs, off = [], 0
    for n in lens:
        probs.append([off, n, off, n, off])
        off += n
    pt = torch.tensor(probs, dtype=torch.int32, device=dev)
    errs = {}
    for dt in (torch.float16, torch.bfloat16):
        d = qkv.to(dt).to(dev)
        q = (d[:, :D].float() * ops.Q_LOG2_SCALE).to(dt) if prescaled else d[:, :D]
        for odt in (dt, torch.float16 if dt == torch.bfloat16 else torch.bfloat16):
            out = torch.zeros(T, D, device=dev, dtype=odt)
            ops.attention(q, d[:, D:2 * D], d[:, 2 * D:], out, pt, max(lens), H, q_prescaled=prescaled)
            o = out.float().cpu()
            off, tot = 0, []
            for n in lens:
                sl = slice(off, off + n)
                qref = q[sl].float().cpu() / (ops.Q_LOG2_SCALE if prescaled else 1.0)
                ref = _ref_attn(qref, d[sl, D:2 * D].float().cpu(), d[sl, 2 * D:].float().cpu(), H)
                tot.append(relerr(o[sl], ref))
                off += n
            errs[(dt, odt)] = max(tot)
    assert errs[(torch.float16, torch.float16)] < 2e-3, errs
    assert errs[(torch.float16, torch.bfloat16)] < 6e-3, errs
    assert errs[(torch.bfloat16, torch.bfloat16)] < 6e-3, errs
    assert errs[(torch.float16, torch.float16)] < errs[(torch.bfloat16, torch.bfloat16)], errs


def test_attention_f16_operands_bench_shape():
    """fp16 q/k/v at the stage-1 bench shape (S = 5,649, 8 heads, the cost-balanced schedule over the full grid:
    every one of the 184 units cut), sampled rows vs fp64."""
    ops = _ops()
    H, S = 8, 5649
    D = H * 128
    g = torch.Generator(device="cpu").manual_seed(5649)
    qkv = torch.randn(S, 3 * D, generator=g).half()
    d = qkv.to(dev)
    probs = [[0, S, 0, S, 0]]
    out = torch.zeros(S, D, device=dev, dtype=torch.float16)
    ops.attention(d[:, :D], d[:, D:2 * D], d[:, 2 * D:], out, torch.tensor(probs, dtype=torch.int32, device=dev), S, H,
                  schedule=ops.attn_schedule(probs, H, dev))
    torch.cuda.synchronize()
    assert _lib_mod().rf_device_error() == 0
    rows = torch.cat([torch.arange(0, 16), torch.randperm(S, generator=g)[:496].sort().values, torch.tensor([S - 1])])
    ref = _ref_attn(qkv[rows, :D].float(), qkv[:, D:2 * D].float(), qkv[:, 2 * D:].float(), H)
    assert relerr(out.float().cpu()[rows], ref) < 2e-3


@pytest.mark.parametrize("sched", [False, True])
def test_attention_stream_k_many_problems(sched):
    """A batch of scenes of very different lengths (batch_infer form): 24 problems, 8 heads, the
    flattened space crossing problem boundaries inside workgroup ranges (equal tile counts, or the
    cost-balanced ranges of rf_attn_schedule)."""
    ops = _ops()
    H = 8
    D = H * 128
    g = torch.Generator(device="cpu").manual_seed(11)
    lens = [int(x) for x in torch.randint(1, 700, (24,), generator=g)]
    T = sum(lens)
    qkv = torch.randn(T, 3 * D, generator=g).bfloat16()
    probs, off = [], 0
    for n in lens:
        probs.append([off, n, off, n, off])
        off += n
    d = qkv.to(dev)
    out = torch.zeros(T, D, device=dev, dtype=torch.bfloat16)
    ops.attention(d[:, :D], d[:, D:2 * D], d[:, 2 * D:], out, torch.tensor(probs, dtype=torch.int32, device=dev),
                  max(lens), H, schedule=ops.attn_schedule(probs, H, dev) if sched else None)
    o = out.float().cpu()
    off = 0
    for n in lens:
        sl = slice(off, off + n)
        ref = _ref_attn(qkv[sl, :D].float(), qkv[sl, D:2 * D].float(), qkv[sl, 2 * D:].float(), H)
        assert relerr(o[sl], ref) < 6e-3, n
        off += n


@pytest.mark.parametrize("sk_kernel_name", ["sk", "p4"])
def test_attention_longest_example_sequence(sk_kernel_name, monkeypatch):
    """S = 11,819 (cbox-lucy: 11,803 triangles + 16 register tokens, the longest example scene; SURVEY §5 needs
    S ~ 12k in one pass) at the model's 8 heads, pre-scaled q, with the cost-balanced schedule: 376 units of
    185 key tiles cut over 256 workgroups.  Checked against fp64 on 768 sampled query rows of every head."""
    if sk_kernel_name == "p4":
        needs_study("the one-wave-per-SIMD attention")
    monkeypatch.setenv("RF_ATTN_P4", "1" if sk_kernel_name == "p4" else "0")
    ops = _ops()
    H, S = 8, 11819
    D = H * 128
    g = torch.Generator(device="cpu").manual_seed(11819)
    qkv = torch.randn(S, 3 * D, generator=g).bfloat16()
    d = qkv.to(dev)
    qs = (d[:, :D].float() * ops.Q_LOG2_SCALE).bfloat16()
    probs = [[0, S, 0, S, 0]]
    out = torch.zeros(S, D, device=dev, dtype=torch.bfloat16)
    ops.attention(qs, d[:, D:2 * D], d[:, 2 * D:], out, torch.tensor(probs, dtype=torch.int32, device=dev), S, H,
                  q_prescaled=True, schedule=ops.attn_schedule(probs, H, dev))
    torch.cuda.synchronize()
    assert _lib_mod().rf_device_error() == 0
    rows = torch.cat([torch.arange(0, 16), torch.randperm(S, generator=g)[:736].sort().values, torch.tensor([S - 1])])
    qref = qs[rows].float().cpu() / ops.Q_LOG2_SCALE
    ref = _ref_attn(qref, qkv[:, D:2 * D].float(), qkv[:, 2 * D:].float(), H)
    assert relerr(out.float().cpu()[rows], ref) < 6e-3


def _lib_mod():
    from renderformer_amd import _lib
    return _lib.load()


def test_attention_bad_schedule_is_refused_and_recovers():
    """A range table built for another launch: the kernel checks it against its own problems instead
    of reading past them, reports a device error (DeviceError at the next call), and after
    ops.clear_device_error() the next launches on fresh workspaces are correct again."""
    from renderformer_amd._lib import DeviceError
    ops = _ops()
    H = 2
    D = H * 128
    g = torch.Generator(device="cpu").manual_seed(3)
    qkv = torch.randn(900, 3 * D, generator=g).bfloat16()
    d = qkv.to(dev)
    small = [[0, 600, 0, 600, 0]]
    big = [[0, 900, 0, 900, 0]]
    wrong = ops.attn_schedule(big, H, dev)  # covers more tiles than the `small` launch has
    out = torch.zeros(900, D, device=dev, dtype=torch.bfloat16)
    ops.attention(d[:, :D], d[:, D:2 * D], d[:, 2 * D:], out, torch.tensor(small, dtype=torch.int32, device=dev), 600, H,
                  schedule=wrong)
    torch.cuda.synchronize()
    assert _lib_mod().rf_device_error() != 0
    with pytest.raises(DeviceError, match="clear_device_error"):
        ops.rmsnorm(torch.ones(4, 256, device=dev), torch.ones(256, device=dev), 1e-6,
                    torch.empty(4, 256, device=dev, dtype=torch.bfloat16))
    ops.clear_device_error()
    assert _lib_mod().rf_device_error() == 0
    for sched in (None, ops.attn_schedule(big, H, dev)):
        out.zero_()
        ops.attention(d[:, :D], d[:, D:2 * D], d[:, 2 * D:], out, torch.tensor(big, dtype=torch.int32, device=dev),
                      900, H, schedule=sched)
        ref = _ref_attn(qkv[:, :D].float(), qkv[:, D:2 * D].float(), qkv[:, 2 * D:].float(), H)
        assert relerr(out.float().cpu(), ref) < 6e-3
    torch.cuda.synchronize()
    assert _lib_mod().rf_device_error() == 0


@pytest.mark.parametrize("grid,shift", [(8, 0), (8, 4), (16, 4), (16, 0)])
def test_swin_attention_matches_oracle_layout(grid, shift):
    ops = _ops()
    H, D, n_img = 2, 256, 2
    T = n_img * grid * grid
    g = torch.Generator(device="cpu").manual_seed(grid + shift)
    q, k, v = [torch.randn(T, D, generator=g).bfloat16() for _ in range(3)]
    out = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
    ops.swin_attention(q.to(dev), k.to(dev), v.to(dev), out, n_img, grid, grid, shift, H)
    # reference: roll, partition, masked SDPA, reverse (attention.py:316-370 with identity projections)
    def part(x):
        x = x.float().view(n_img, grid, grid, D)
        if shift:
            x = torch.roll(x, (-shift, -shift), (1, 2))
        return x.view(n_img, grid // 8, 8, grid // 8, 8, D).permute(0, 1, 3, 2, 4, 5).reshape(-1, 64, H, 128).transpose(1, 2)
    qw, kw, vw = part(q), part(k), part(v)
    mask = rf_ref.swin_mask(grid, grid, 8, shift).repeat(n_img, 1, 1)[:, None] if shift else None
    o = F.scaled_dot_product_attention(qw.double(), kw.double(), vw.double(), attn_mask=mask)
    o = o.transpose(1, 2).reshape(n_img, grid // 8, grid // 8, 8, 8, D).permute(0, 1, 3, 2, 4, 5).reshape(n_img, grid, grid, D)
    if shift:
        o = torch.roll(o, (shift, shift), (1, 2))
    assert relerr(out.float().cpu(), o.reshape(T, D)) < 6e-3


def test_prologue_kernels_match_oracle():
    ops = _ops()
    from renderformer_amd.scenes import batch_scenes, synthetic_scene
    scenes = [synthetic_scene(40, 2, seed=3), synthetic_scene(25, 2, seed=4)]
    bt = batch_scenes(scenes, padding_length=48)
    B, N = 2, 48
    mask = bt["mask"]
    valid = torch.nonzero(mask.reshape(-1)).squeeze(1).int()
    dst = torch.full((B * N,), -1, dtype=torch.int32)
    dst[valid.long()] = torch.arange(valid.numel(), dtype=torch.int32)
    # texture: in-place log encode of every row + packed bf16 of valid rows
    tex = bt["texture"].clone().to(dev)
    out = torch.empty(valid.numel(), 13 * 1024, device=dev, dtype=torch.bfloat16)
    ops.texture_pack(tex, 3, dst.to(dev), out)
    ref = bt["texture"].clone()
    ref[:, :, -3:] = torch.log10(ref[:, :, -3:] + 1)
    assert torch.allclose(tex.cpu(), ref, rtol=1e-6, atol=1e-6)
    assert torch.equal(out.cpu(), ref.reshape(B * N, -1)[valid.long()].bfloat16())
    # vn NeRF encoding
    vo = torch.empty(valid.numel(), 128, device=dev, dtype=torch.bfloat16)
    ops.vn_encode(bt["vn"].reshape(B, N, 9).contiguous().to(dev), dst.to(dev), 6, vo)
    refv = rf_ref.nerf_encode(bt["vn"].reshape(B * N, 9)[valid.long()], 6)
    assert torch.allclose(vo[:, :117].float().cpu(), refv.bfloat16().float(), atol=1e-2)
    assert (vo[:, 117:] == 0).all()
    # rays (+ patchify) vs RayGenerator restatement
    res, P = 64, 4
    c2w = bt["c2w"].reshape(P, 4, 4).contiguous()
    fov = bt["fov"].reshape(P).contiguous()
    ro, rd = rf_ref.ray_gen(c2w, fov[:, None] / 180.0 * torch.pi, res)
    tok = torch.empty(P * 64, 192, device=dev, dtype=torch.bfloat16)
    rpos = torch.empty(P, 9, device=dev)
    ops.ray_tokens(c2w.to(dev), fov.to(dev), res, 8, tok, rpos)
    reft = rd.view(P, 8, 8, 8, 8, 3).permute(0, 1, 3, 5, 2, 4).reshape(P * 64, 192)
    assert (tok.float().cpu() - reft.bfloat16().float()).abs().max() < 1e-2
    assert torch.allclose(rpos.cpu(), ro.repeat(1, 3))
    tok2 = torch.empty_like(tok)
    ops.patchify_rays(rd.contiguous().to(dev), 8, tok2)
    assert torch.equal(tok2.cpu(), reft.bfloat16())
    # RoPE positions: camera transform + register-token centre
    counts = mask.sum(1).tolist()
    scene_off = torch.tensor([0, counts[0], counts[0] + counts[1]], dtype=torch.int32)
    S = [16 + c for c in counts]
    set_off = torch.tensor([0, S[0], 2 * S[0], 2 * S[0] + S[1], 2 * S[0] + 2 * S[1]], dtype=torch.int32)
    pos = torch.empty(int(set_off[-1]), 9, device=dev)
    ops.scene_pos(bt["triangles"].reshape(B * N, 9).contiguous().to(dev), valid.to(dev), scene_off.to(dev),
                  c2w.to(dev), B, 2, 16, pos, set_off.to(dev), max(counts))
    tcam = rf_ref.cam_transform(c2w, torch.repeat_interleave(bt["triangles"], 2, 0)).reshape(P, N, 9)
    refp, _ = rf_ref.center_pos(tcam, torch.repeat_interleave(mask, 2, 0), 16)
    for p in range(P):
        n = counts[p // 2]
        got = pos[int(set_off[p]):int(set_off[p + 1])].cpu()
        assert torch.allclose(got, refp[p, :16 + n], atol=2e-6), p


def test_scene_pos_large_and_deterministic():
    """Two-launch positions / centres on cbox-lucy-sized scenes (47 blocks of 256 triangles, ragged): vs the
    oracle, and bit-identical run to run (block partials reduced in a fixed order, no atomics)."""
    from oracle import rf_ref
    from renderformer_amd.scenes import batch_scenes, synthetic_scene
    ops = _ops()
    counts = [11803, 5000]
    bt = batch_scenes([synthetic_scene(n, 1, seed=40 + i) for i, n in enumerate(counts)], expand=False)
    B, N = bt["mask"].shape
    valid = torch.nonzero(bt["mask"].reshape(-1)).squeeze(1).to(torch.int32)
    scene_off = torch.tensor([0, counts[0], sum(counts)], dtype=torch.int32)
    S = [16 + c for c in counts]
    set_off = torch.tensor([0, S[0], S[0] + S[1]], dtype=torch.int32)
    tris = bt["triangles"].reshape(B * N, 9).contiguous()
    outs = []
    for _ in range(2):
        pos = torch.empty(sum(S), 9, device=dev)
        ops.scene_pos(tris.to(dev), valid.to(dev), scene_off.to(dev), None, B, 1, 16, pos, set_off.to(dev), max(counts))
        outs.append(pos.cpu())
    assert torch.equal(outs[0], outs[1])
    refp, _ = rf_ref.center_pos(bt["triangles"].reshape(B, N, 9), bt["mask"], 16)
    for b in range(B):
        got = outs[0][int(set_off[b]):int(set_off[b + 1])]
        assert torch.allclose(got, refp[b, :S[b]], atol=2e-6), b


def test_scene_pos_undersized_max_tris_reports_device_error():
    """max_tris below a set's triangle count: the centre kernel stays inside its set's partial slots
    and raises device error 4 instead of reading the next set's sums; clear_device_error() recovers."""
    from renderformer_amd._lib import DeviceError
    from renderformer_amd.scenes import batch_scenes, synthetic_scene
    ops = _ops()
    counts = [700, 300]
    bt = batch_scenes([synthetic_scene(n, 1, seed=50 + i) for i, n in enumerate(counts)], expand=False)
    B, N = bt["mask"].shape
    valid = torch.nonzero(bt["mask"].reshape(-1)).squeeze(1).to(torch.int32).to(dev)
    scene_off = torch.tensor([0, counts[0], sum(counts)], dtype=torch.int32, device=dev)
    S = [16 + c for c in counts]
    set_off = torch.tensor([0, S[0], S[0] + S[1]], dtype=torch.int32, device=dev)
    tris = bt["triangles"].reshape(B * N, 9).contiguous().to(dev)
    pos = torch.zeros(sum(S), 9, device=dev)
    ops.scene_pos(tris, valid, scene_off, None, B, 1, 16, pos, set_off, 300)  # 300 < 700: 2 blocks, not 3
    torch.cuda.synchronize()
    assert _lib_mod().rf_device_error() == 4
    with pytest.raises(DeviceError, match="clear_device_error"):
        ops.scene_pos(tris, valid, scene_off, None, B, 1, 16, pos, set_off, max(counts))
    ops.clear_device_error()
    ops.scene_pos(tris, valid, scene_off, None, B, 1, 16, pos, set_off, max(counts))
    torch.cuda.synchronize()
    assert _lib_mod().rf_device_error() == 0
    refp, _ = rf_ref.center_pos(bt["triangles"].reshape(B, N, 9), bt["mask"], 16)
    for b in range(B):
        assert torch.allclose(pos[int(set_off[b]):int(set_off[b + 1])].cpu(), refp[b, :S[b]], atol=2e-6), b


def test_hdr_output():
    ops = _ops()
    logits = torch.randn(2, 3, 16, 16, device=dev)
    out = torch.empty(2, 16, 16, 3, device=dev)
    ops.hdr_output(logits, out, 1e-3, True)
    ref = torch.pow(10.0, F.elu(logits, 1e-3).permute(0, 2, 3, 1)) - 1
    assert torch.allclose(out, ref, rtol=1e-6, atol=1e-6)


# ----------------------------------------------------------------------------- DPT convolutions
# bf16x3 is checked against fp64 at fp32-level accuracy; f16 against fp64 convolutions of the
# fp16-ROUNDED operands (what one fp16 MFMA with fp32 accumulation computes exactly, up to the sum order).
PRECS = ["bf16x3", "f16"]


def _q(t, prec):
    """fp64 copy of an operand as the kernel sees it."""
    return t.double() if prec == "bf16x3" else t.half().double()


def _planes_value(pl):
    return pl.hi.float() if pl.f16 else pl.hi.float() + pl.lo.float()


@pytest.mark.parametrize("tile", ["auto", "4w", "64", "6412", "6464"])
@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("cin,cout,k,stride,hw", [(64, 128, 3, 1, 17), (256, 256, 3, 1, 32), (16, 32, 3, 1, 20),
                                                   (1024, 128, 1, 1, 16), (128, 128, 3, 2, 16), (48, 200, 3, 1, 9)])
def test_conv_matches_fp64(cin, cout, k, stride, hw, prec, tile, monkeypatch):
    """auto: small grids on the 8-wave 128x128 tile (data-parallel or stream-K); 4w: the 4-wave tile; 64 / 6412:
    the data-parallel 64x64 / 64x128 small-level tiles, 6464: stream-K over the 64x64 tile (fp16 only)."""
    if tile in ("64", "6412", "6464") and prec != "f16":
        pytest.skip("the small-level tiles serve fp16 operands")
    if tile == "4w":
        monkeypatch.setenv("RF_CONV_SKW8", "0")
        monkeypatch.setenv("RF_CONV_TILE", "128")
    elif tile != "auto":
        monkeypatch.setenv("RF_CONV_TILE", tile)
    from renderformer_amd.dpt import _Conv, split_planes
    f16 = prec == "f16"
    g = torch.Generator(device="cpu").manual_seed(cin + cout)
    w = torch.randn(cout, cin, k, k, generator=g) / math.sqrt(cin * k * k)
    b = torch.randn(cout, generator=g)
    x = torch.randn(2, cin, hw, hw, generator=g)
    conv = _Conv(w, b, dev, f16=f16)
    xn = x.permute(0, 2, 3, 1).contiguous().to(dev)
    pad = k // 2
    ref = F.conv2d(_q(x, prec), _q(w, prec), b.double(), stride=stride, padding=pad).permute(0, 2, 3, 1)
    out, _ = conv(split_planes(xn, conv.cin_pad, f16=f16), stride=stride, pad=pad, out_f32=True)
    assert relerr(out.cpu(), ref) < 2e-5
    if f16:  # and the fp16 rounding itself stays small against the exact fp64 convolution
        exact = F.conv2d(x.double(), w.double(), b.double(), stride=stride, padding=pad).permute(0, 2, 3, 1)
        assert relerr(out.cpu(), exact) < 1e-3
    if stride == 1 and k == 3 and cin == cout:
        r1 = torch.randn(ref.shape, generator=g)
        r2 = torch.randn(ref.shape, generator=g)
        out, pl = conv(split_planes(xn, conv.cin_pad, silu=True, f16=f16), res1=r1.to(dev), res2=r2.to(dev),
                       out_f32=True, planes_ld=cout + 32, planes_silu=True)
        sx = _q(F.silu(x.double()).float(), prec)
        ref2 = F.conv2d(sx, _q(w, prec), b.double(), padding=pad).permute(0, 2, 3, 1) + r1 + r2
        assert relerr(out.cpu(), ref2) < 2e-5
        assert relerr(_planes_value(pl)[..., :cout].cpu(), F.silu(ref2)) < (1e-3 if f16 else 2e-5)
        assert (pl.hi[..., cout:] == 0).all() and (f16 or (pl.lo[..., cout:] == 0).all())


@pytest.mark.parametrize("tile", ["128", "1288", "256", "64"])
@pytest.mark.parametrize("cin,cout,hw", [(256, 256, 32), (64, 128, 64), (32, 256, 16), (128, 128, 128),
                                         (64, 256, 256), (128, 32, 64), (64, 32, 256)])
def test_conv_halo(cin, cout, hw, tile, monkeypatch):
    """Halo-tiled 3x3 convolution (RF_CONV_HALO=1) on every tile that takes it: tiles of whole image rows
    (TW = wo) and of partial rows (TW = BM), two images, fused bias + 2 residuals + SiLU planes.  Tile "64"
    is the 256x64 tile every filter bank of <= 64 channels takes (DPT output_conv2)."""
    if tile == "256" and cout % 256:
        pytest.skip("256x256 tile needs 256 output channels")
    if (tile == "64") != (cout <= 64):
        pytest.skip("the 256x64 tile serves exactly the filter banks of <= 64 channels")
    monkeypatch.setenv("RF_CONV_HALO", "1")
    monkeypatch.setenv("RF_CONV_TILE", tile)
    monkeypatch.setenv("RF_CONV_SK", "0")
    from renderformer_amd.dpt import _Conv, split_planes
    g = torch.Generator(device="cpu").manual_seed(cin * hw + cout)
    w = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(cin * 9)
    b = torch.randn(cout, generator=g)
    x = torch.randn(2, cin, hw, hw, generator=g)
    conv = _Conv(w, b, dev, f16=True)
    xn = x.permute(0, 2, 3, 1).contiguous().to(dev)
    r1 = torch.randn(2, hw, hw, cout, generator=g)
    r2 = torch.randn(2, hw, hw, cout, generator=g)
    out, pl = conv(split_planes(xn, conv.cin_pad, silu=True, f16=True), res1=r1.to(dev), res2=r2.to(dev),
                   out_f32=True, planes_ld=cout, planes_silu=True)
    sx = _q(F.silu(x.double()).float(), "f16")
    ref = F.conv2d(sx, _q(w, "f16"), b.double(), padding=1).permute(0, 2, 3, 1) + r1 + r2
    assert relerr(out.cpu(), ref) < 2e-5
    assert relerr(_planes_value(pl)[..., :cout].cpu(), F.silu(ref)) < 1e-3


@pytest.mark.parametrize("h2s", ["3", "4", "5"])
@pytest.mark.parametrize("cin,cout,hh,ww,n_img", [(256, 128, 32, 64, 2), (128, 256, 48, 32, 1), (32, 128, 16, 32, 3),
                                                  (96, 128, 16, 96, 1), (256, 256, 64, 64, 1), (128, 32, 32, 64, 2),
                                                  (64, 64, 16, 32, 1)])
def test_conv_halo2(cin, cout, hh, ww, n_img, h2s, monkeypatch):
    """The 16 x 32-pixel halo-tiled 3x3 convolution (halo2_kernel; forced on with RF_CONV_HALO2=1, it is the
    default at the 512^2 / 256^2 DPT levels): 1, 2, 3, 4 and 8 channel chunks (the next chunk's halo issued under
    the current one), several images and tiles along both axes, non-square images, both W ring depths, the
    128-channel block (1 or 2 channel tiles) and the 64-channel block (32 and 64 output channels), fused
    bias + 2 residuals + SiLU fp16 planes with a padded row stride."""
    monkeypatch.setenv("RF_CONV_HALO2", "1")
    monkeypatch.setenv("RF_CONV_HALO3", "0")
    monkeypatch.setenv("RF_CONV_HK", "0")
    monkeypatch.setenv("RF_CONV_H2S", h2s)
    from renderformer_amd.dpt import _Conv, split_planes
    g = torch.Generator(device="cpu").manual_seed(cin * hh + cout + ww)
    w = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(cin * 9)
    b = torch.randn(cout, generator=g)
    x = torch.randn(n_img, cin, hh, ww, generator=g)
    conv = _Conv(w, b, dev, f16=True)
    xn = x.permute(0, 2, 3, 1).contiguous().to(dev)
    r1 = torch.randn(n_img, hh, ww, cout, generator=g)
    r2 = torch.randn(n_img, hh, ww, cout, generator=g)
    out, pl = conv(split_planes(xn, conv.cin_pad, silu=True, f16=True), res1=r1.to(dev), res2=r2.to(dev),
                   out_f32=True, planes_ld=cout + 32, planes_silu=True)
    sx = _q(F.silu(x.double()).float(), "f16")
    ref = F.conv2d(sx, _q(w, "f16"), b.double(), padding=1).permute(0, 2, 3, 1) + r1 + r2
    assert relerr(out.cpu(), ref) < 2e-5
    assert relerr(_planes_value(pl)[..., :cout].cpu(), F.silu(ref)) < 1e-3
    assert (pl.hi[..., cout:] == 0).all()
    # plain output (no residuals): the same kernel against the unfused conv
    out2, _ = conv(split_planes(xn, conv.cin_pad, f16=True), out_f32=True)
    ref2 = F.conv2d(_q(x, "f16"), _q(w, "f16"), b.double(), padding=1).permute(0, 2, 3, 1)
    assert relerr(out2.cpu(), ref2) < 2e-5


@pytest.mark.parametrize("cin,cout,hh,ww,n_img", [(256, 128, 32, 64, 2), (128, 256, 48, 32, 1), (32, 128, 16, 32, 3),
                                                  (96, 128, 16, 96, 1), (256, 256, 64, 64, 1), (64, 384, 16, 32, 1),
                                                  (512, 128, 16, 32, 1)])
def test_conv_halo3(cin, cout, hh, ww, n_img, monkeypatch):
    """halo3_kernel (the default for the 512^2 / 256^2 DPT convs with a multiple of 128 filters: the bank read from L2
    into a register ring, one barrier per 32-channel chunk): 1 to 16 channel chunks (the last chunk re-stages its own
    halo and the last taps re-load the last W slice), several images, tiles along both axes, 1 to 3 channel tiles,
    fused bias + 2 residuals + SiLU fp16 planes with a padded row stride, and the plain fp32 output; against fp64 on
    the same fp16 operands and against halo2 (same products, fp32 summation order)."""
    monkeypatch.setenv("RF_CONV_HALO2", "1")
    monkeypatch.setenv("RF_CONV_HALO3", "1")
    from renderformer_amd.dpt import _Conv, split_planes
    g = torch.Generator(device="cpu").manual_seed(cin * hh + cout + ww + 11)
    w = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(cin * 9)
    b = torch.randn(cout, generator=g)
    x = torch.randn(n_img, cin, hh, ww, generator=g)
    conv = _Conv(w, b, dev, f16=True)
    xn = x.permute(0, 2, 3, 1).contiguous().to(dev)
    r1 = torch.randn(n_img, hh, ww, cout, generator=g)
    r2 = torch.randn(n_img, hh, ww, cout, generator=g)
    out, pl = conv(split_planes(xn, conv.cin_pad, silu=True, f16=True), res1=r1.to(dev), res2=r2.to(dev),
                   out_f32=True, planes_ld=cout + 32, planes_silu=True)
    sx = _q(F.silu(x.double()).float(), "f16")
    ref = F.conv2d(sx, _q(w, "f16"), b.double(), padding=1).permute(0, 2, 3, 1) + r1 + r2
    assert relerr(out.cpu(), ref) < 2e-5
    assert relerr(_planes_value(pl)[..., :cout].cpu(), F.silu(ref)) < 1e-3
    assert (pl.hi[..., cout:] == 0).all()
    out2, _ = conv(split_planes(xn, conv.cin_pad, f16=True), out_f32=True)
    ref2 = F.conv2d(_q(x, "f16"), _q(w, "f16"), b.double(), padding=1).permute(0, 2, 3, 1)
    assert relerr(out2.cpu(), ref2) < 2e-5
    monkeypatch.setenv("RF_CONV_HALO3", "0")  # halo2 on the same operands
    out3, _ = conv(split_planes(xn, conv.cin_pad, f16=True), out_f32=True)
    assert relerr(out3.cpu(), out2.cpu().double()) < 1e-6


@pytest.mark.parametrize("cin,cout,hh,ww,n_img", [(256, 128, 32, 64, 2), (128, 256, 48, 32, 1), (32, 64, 16, 32, 3),
                                                  (96, 128, 16, 96, 1), (256, 256, 64, 64, 1), (64, 192, 16, 32, 1)])
def test_conv_hk(cin, cout, hh, ww, n_img, monkeypatch):
    """conv3x3_hk_kernel (forced on with RF_CONV_HK=1; the default for the 512^2 / 256^2 DPT convs with >= 256 blocks):
    1 to 8 channel chunks, several images, tiles along both axes, 1 to 4 channel tiles of 64, fused bias + 2
    residuals + SiLU fp16 planes with a padded row stride, and the plain fp32 output; against fp64 on the same fp16
    operands and against the halo2 kernel (same products, fp32 summation order)."""
    needs_study("conv3x3_hk_kernel")
    monkeypatch.setenv("RF_CONV_HK", "1")
    from renderformer_amd.dpt import _Conv, split_planes
    g = torch.Generator(device="cpu").manual_seed(cin * hh + cout + ww + 7)
    w = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(cin * 9)
    b = torch.randn(cout, generator=g)
    x = torch.randn(n_img, cin, hh, ww, generator=g)
    conv = _Conv(w, b, dev, f16=True)
    xn = x.permute(0, 2, 3, 1).contiguous().to(dev)
    r1 = torch.randn(n_img, hh, ww, cout, generator=g)
    r2 = torch.randn(n_img, hh, ww, cout, generator=g)
    out, pl = conv(split_planes(xn, conv.cin_pad, silu=True, f16=True), res1=r1.to(dev), res2=r2.to(dev),
                   out_f32=True, planes_ld=cout + 32, planes_silu=True)
    sx = _q(F.silu(x.double()).float(), "f16")
    ref = F.conv2d(sx, _q(w, "f16"), b.double(), padding=1).permute(0, 2, 3, 1) + r1 + r2
    assert relerr(out.cpu(), ref) < 2e-5
    assert relerr(_planes_value(pl)[..., :cout].cpu(), F.silu(ref)) < 1e-3
    assert (pl.hi[..., cout:] == 0).all()
    out2, _ = conv(split_planes(xn, conv.cin_pad, f16=True), out_f32=True)
    ref2 = F.conv2d(_q(x, "f16"), _q(w, "f16"), b.double(), padding=1).permute(0, 2, 3, 1)
    assert relerr(out2.cpu(), ref2) < 2e-5
    if cout % 128 == 0:  # the halo2 kernel on the same operands
        monkeypatch.setenv("RF_CONV_HK", "0")
        monkeypatch.setenv("RF_CONV_HALO2", "1")
        monkeypatch.setenv("RF_CONV_HALO3", "0")
        out3, _ = conv(split_planes(xn, conv.cin_pad, f16=True), out_f32=True)
        assert relerr(out3.cpu(), out2.cpu().double()) < 1e-6


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("cin,cout,k", [(128, 128, 4), (256, 256, 2), (16, 16, 4), (32, 32, 2)])
def test_deconv(cin, cout, k, prec):
    from renderformer_amd.dpt import _Conv, split_planes
    f16 = prec == "f16"
    g = torch.Generator(device="cpu").manual_seed(k * cin)
    w = torch.randn(cin, cout, k, k, generator=g) / math.sqrt(cin)
    b = torch.randn(cout, generator=g)
    x = torch.randn(2, cin, 8, 8, generator=g)
    conv = _Conv(w, b, dev, deconv=True, f16=f16)
    xs = split_planes(x.permute(0, 2, 3, 1).contiguous().to(dev), conv.cin_pad, f16=f16)
    out, _ = conv(xs, out_f32=True)
    ref = F.conv_transpose2d(_q(x, prec), _q(w, prec), b.double(), stride=k).permute(0, 2, 3, 1)
    assert relerr(out.cpu(), ref) < 2e-5
    out2, pl = conv(xs, planes_ld=cout)  # plane output only
    assert out2 is None and relerr(_planes_value(pl).cpu(), ref) < (1e-3 if f16 else 2e-5)


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("c", [12, 16])  # 4- and 8-channel-per-thread kernels
@pytest.mark.parametrize("hi,ho", [(8, 16), (16, 32), (32, 64), (7, 13)])
def test_upsample_bilinear_align_corners(hi, ho, c, prec):
    from renderformer_amd.dpt import upsample
    f16 = prec == "f16"
    x = torch.randn(2, c, hi, hi)
    out, pl = upsample(x.permute(0, 2, 3, 1).contiguous().to(dev), ho, ho, planes_ld=32, f16=f16)
    ref = F.interpolate(x, size=(ho, ho), mode="bilinear", align_corners=True).permute(0, 2, 3, 1)
    assert torch.allclose(out.cpu(), ref, atol=1e-5, rtol=1e-5)
    if f16:
        assert torch.equal(pl.hi[..., :c].cpu(), out.cpu().half())  # RNE fp16 of the fp32 value
        assert (pl.hi[..., c:] == 0).all()
    else:
        assert torch.allclose(_planes_value(pl)[..., :c].cpu(), ref, atol=1e-5, rtol=1e-5)
    # plane-only output (the DPT's last upsample) equals the planes written alongside the fp32 output
    out2, pl2 = upsample(x.permute(0, 2, 3, 1).contiguous().to(dev), ho, ho, out_f32=False, planes_ld=32, f16=f16)
    assert out2 is None and torch.equal(pl2.hi, pl.hi) and (f16 or torch.equal(pl2.lo, pl.lo))


@pytest.mark.parametrize("hi,ho,c,ld_in,ld_out", [(4, 9, 16, 16, 32), (256, 512, 256, 256, 256), (33, 64, 40, 48, 40)])
def test_upsample_planes_f16_in(hi, ho, c, ld_in, ld_out):
    """rf_upsample_bilinear_h (fp16 planes in and out, the folded DPT tail): the fp32 blend of the plane's
    fp16 values rounded once, vs F.interpolate on the same values; padded channels stay zero."""
    from renderformer_amd.dpt import Planes, upsample_planes
    g = torch.Generator(device="cpu").manual_seed(hi + c)
    x = torch.randn(2, hi, hi, c, generator=g).half()
    pin = Planes.empty(2, hi, hi, c, ld_in, dev, True)
    pin.hi[..., :c] = x.to(dev)
    pl = upsample_planes(pin, ho, ho, planes_ld=ld_out)
    ref = F.interpolate(x.float().permute(0, 3, 1, 2), size=(ho, ho), mode="bilinear",
                        align_corners=True).permute(0, 2, 3, 1)
    got = pl.hi[..., :c].float().cpu()
    assert float((got - ref).abs().max()) <= float(ref.abs().max()) * 2.0 ** -10  # one fp16 rounding
    assert relerr(got, ref) < 4e-4
    assert (pl.hi[..., c:] == 0).all()


def test_conv1x1_group_matches_single_convs():
    """rf_conv1x1_f16_group (the DPT tap projections as one launch) vs the fp64 convolution of each, and vs
    one rf_conv2d_f16 call each; one conv without bias."""
    from renderformer_amd.dpt import _Conv, conv1x1_group, split_planes
    g = torch.Generator(device="cpu").manual_seed(3)
    couts, cin, hw = (128, 256, 512, 1024), 1024, 24
    convs, xs, refs = [], [], []
    for q, co in enumerate(couts):
        w = torch.randn(co, cin, 1, 1, generator=g) / 32
        b = None if q == 2 else torch.randn(co, generator=g)
        x = torch.randn(1, cin, hw, hw, generator=g)
        conv = _Conv(w, b, dev, f16=True)
        convs.append(conv)
        xs.append(split_planes(x.permute(0, 2, 3, 1).contiguous().to(dev), conv.cin_pad, f16=True))
        refs.append(F.conv2d(_q(x, "f16"), _q(w, "f16"), None if b is None else b.double()).permute(0, 2, 3, 1))
    lds = [c + 32 for c in couts]
    outs = conv1x1_group(convs, xs, lds)
    for conv, x, o, ref, ld in zip(convs, xs, outs, refs, lds):
        assert o.shape[-1] == ld and (o.hi[..., conv.cout:] == 0).all()
        assert relerr(o.hi[..., :conv.cout].float().cpu(), ref) < 1e-3
        _, single = conv(x, planes_ld=ld)
        assert relerr(o.hi.float(), single.hi.float()) < 1e-3
    bad = split_planes(torch.randn(1, hw, hw, 512, device=dev), 512, f16=True)  # wrong channel count
    with pytest.raises(ValueError):
        conv1x1_group(convs[:2], [xs[0], bad], lds[:2])


def test_conv_group_matches_single_launches():
    """rf_conv2d_f16_group: a deconvolution (k = 4), a stride-2 3x3 convolution with bias, and two 3x3
    convolutions of different sizes with fp32 + SiLU-plane outputs in one launch, each vs its own launch."""
    from renderformer_amd.dpt import _Conv, conv_group, split_planes
    g = torch.Generator(device="cpu").manual_seed(4)

    def planes(c, hw):
        return split_planes(torch.randn(1, hw, hw, c, generator=g).to(dev), c, f16=True)

    dec = _Conv(torch.randn(64, 128, 4, 4, generator=g) / 16, torch.randn(128, generator=g), dev, deconv=True, f16=True)
    s2 = _Conv(torch.randn(128, 96, 3, 3, generator=g) / 30, torch.randn(128, generator=g), dev, f16=True)
    c1 = _Conv(torch.randn(256, 64, 3, 3, generator=g) / 24, None, dev, f16=True)
    c2 = _Conv(torch.randn(256, 256, 3, 3, generator=g) / 48, None, dev, f16=True)
    jobs = [dict(conv=dec, x=planes(64, 12), planes_ld=128),
            dict(conv=s2, x=planes(96, 20), stride=2, pad=1, planes_ld=160),
            dict(conv=c1, x=planes(64, 24), out_f32=True, planes_ld=256, planes_silu=True),
            dict(conv=c2, x=planes(256, 9), out_f32=True, planes_ld=256, planes_silu=True)]
    got = conv_group(jobs)
    for j, (out, pl) in zip(jobs, got):
        kw = {k: v for k, v in j.items() if k not in ("conv", "x")}
        if j["conv"].k:
            kw.pop("stride", None), kw.pop("pad", None)
        ref_out, ref_pl = j["conv"](j["x"], **kw)
        assert relerr(pl.hi.float(), ref_pl.hi.float()) < 1e-3
        if out is not None:
            assert relerr(out, ref_out) < 1e-5
    with pytest.raises(ValueError):
        conv_group([dict(conv=c2, x=planes(64, 9))])  # input planes of the wrong width


@pytest.mark.parametrize("hw,halo2,hk,halo3", [(24, "0", "0", "0"), (64, "1", "0", "0"), (64, "0", "1", "0"),
                                               (64, "1", "0", "1")])
def test_conv_border_bias(hw, halo2, hk, halo3, monkeypatch):
    """RF_CONV_BORDER_BIAS: per-pixel bias row by border class (3 ry + rx), on the engine tile, the halo2, hk and
    halo3 kernels (the folded output_conv1), vs torch conv + the class bias."""
    from renderformer_amd.dpt import _Conv, split_planes
    if hk == "1":
        needs_study("conv3x3_hk_kernel")
    monkeypatch.setenv("RF_CONV_HALO2", halo2)
    monkeypatch.setenv("RF_CONV_HK", hk)
    monkeypatch.setenv("RF_CONV_HALO3", halo3)
    g = torch.Generator(device="cpu").manual_seed(hw)
    cin, cout = 64, 128
    w = torch.randn(cout, cin, 3, 3, generator=g) / 24
    b9 = torch.randn(9, cout, generator=g)
    x = torch.randn(2, cin, hw, hw, generator=g)
    conv = _Conv(w, None, dev, f16=True)
    _, pl = conv(split_planes(x.permute(0, 2, 3, 1).contiguous().to(dev), conv.cin_pad, f16=True), planes_ld=cout,
                 border_bias=b9.to(dev).contiguous())
    ref = F.conv2d(_q(x, "f16"), _q(w, "f16"), None, padding=1)
    ry = torch.ones(hw, dtype=torch.long)
    ry[0], ry[-1] = 0, 2
    ref = (ref + b9.double()[3 * ry[:, None] + ry[None, :]].permute(2, 0, 1)[None]).permute(0, 2, 3, 1)
    assert relerr(pl.hi.float().cpu(), ref) < 1e-3
    with pytest.raises(Exception):  # the flag needs a 3x3 stride-1 pad-1 convolution
        conv(split_planes(x.permute(0, 2, 3, 1).contiguous().to(dev), conv.cin_pad, f16=True), stride=2, pad=1,
             planes_ld=cout, border_bias=b9.to(dev).contiguous())


@pytest.mark.parametrize("prec,hw", [("bf16x3", 24), ("f16", 24), ("f16h2", 32), ("f16h2", 64)])
def test_conv_final_head(prec, hw, monkeypatch):
    """output_conv2 + its fused head (SiLU, 1x1 32 -> 3, ELU, 10^x - 1); f16h2: on the 16 x 32-pixel halo kernel's
    64-channel block (RF_CONV_HALO2=1; the default for 512^2 frames)."""
    from renderformer_amd.dpt import LOG_DECODE, NCHW_OUT, _Conv, split_planes
    if prec == "f16h2":
        monkeypatch.setenv("RF_CONV_HALO2", "1")
        prec = "f16"
    f16 = prec == "f16"
    g = torch.Generator(device="cpu").manual_seed(9)
    w = torch.randn(32, 64, 3, 3, generator=g) / 24
    b = torch.randn(32, generator=g) * 0.1
    wf = torch.randn(3, 32, 1, 1, generator=g) / 6
    bf = torch.randn(3, generator=g) * 0.1
    x = torch.randn(2, 64, hw, hw, generator=g)
    conv = _Conv(w, b, dev, f16=f16)
    y = F.conv2d(F.silu(F.conv2d(_q(x, prec), _q(w, prec), b.double(), padding=1)), wf.double(), bf.double())
    y = F.elu(y, 1e-3)
    xs = split_planes(x.permute(0, 2, 3, 1).contiguous().to(dev), conv.cin_pad, f16=f16)
    fin = (wf.reshape(3, 32).to(dev), bf.to(dev), 1e-3)
    out = conv(xs, final=fin, final_flags=LOG_DECODE)
    assert relerr(out.cpu(), (10 ** y - 1).permute(0, 2, 3, 1)) < 2e-5
    out2 = conv(xs, final=fin, final_flags=NCHW_OUT)
    assert relerr(out2.cpu(), y) < 2e-5


def test_split_planes_f16_rounding():
    from renderformer_amd.dpt import split_planes
    x = torch.randn(3, 5, 7, 20) * 100
    x[0, 0, 0, :4] = torch.tensor([7e4, -7e4, 1e-8, 65504.0])  # overflow -> inf, underflow -> 0, max exact
    pl = split_planes(x.to(dev), 24, f16=True)
    assert pl.hi.dtype == torch.float16 and pl.lo is None
    assert torch.equal(pl.hi[..., :20].cpu(), x.half())
    pl = split_planes(x.to(dev), 24, silu=True, f16=True)
    assert torch.allclose(pl.hi[..., :20].cpu().float(), F.silu(x).half().float(), rtol=1e-3, atol=1e-6)


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("final", [False, True])
def test_conv_stream_k_matches_data_parallel(monkeypatch, final, prec):
    """Few output tiles (the DPT's 32x32 / 64x64 levels): the stream-K split (8 blocks per tile here) must
    agree with the one-block-per-tile launch and with fp64, including residuals, planes and the fused head."""
    from renderformer_amd.dpt import LOG_DECODE, _Conv, split_planes
    g = torch.Generator(device="cpu").manual_seed(77)
    cin = cout = 256 if not final else 64
    w = torch.randn(cout if not final else 32, cin, 3, 3, generator=g) / math.sqrt(cin * 9)
    b = torch.randn(w.shape[0], generator=g)
    x = torch.randn(2, cin, 32, 32, generator=g)
    f16 = prec == "f16"
    conv = _Conv(w, b, dev, f16=f16)
    xs = split_planes(x.permute(0, 2, 3, 1).contiguous().to(dev), conv.cin_pad, silu=True, f16=f16)
    outs = []
    fin = (torch.randn(3, 32, generator=g).to(dev) / 6, torch.zeros(3, device=dev), 1e-3)
    for sk in ("1", "0"):
        monkeypatch.setenv("RF_CONV_SK", sk)
        if final:
            outs.append((conv(xs, final=fin, final_flags=LOG_DECODE), None))
        else:
            r1 = torch.ones(2, 32, 32, cout, device=dev)
            outs.append(conv(xs, res1=r1, out_f32=True, planes_ld=cout, planes_silu=True))
    (a, pa), (bb, pb) = outs
    assert relerr(a, bb) < 1e-6
    if not final:
        sx = _q(F.silu(x.double()).float(), prec)
        ref = F.conv2d(sx, _q(w, prec), b.double(), padding=1).permute(0, 2, 3, 1) + 1.0
        assert relerr(a.cpu(), ref) < 2e-5
        # fp16 planes: a last-bit fp32 difference from the other K split can flip one fp16 rounding
        assert relerr(_planes_value(pa), _planes_value(pb)) < (1e-4 if f16 else 1e-6)


# ----------------------------------------------------------------------------- texture encoder fast path
def _to_h5_texture(b, n, c, seed):
    from renderformer_amd.scenes import texture_mask
    g = torch.Generator(device="cpu").manual_seed(seed)
    const = torch.rand(b, n, c, generator=g) * 4
    return const[..., None, None] * torch.from_numpy(texture_mask(32)).float()


@pytest.mark.parametrize("log_ch", [0, 3])
def test_texture_scan(log_ch):
    """rf_texture_scan: in-place log encode identical to rf_texture_pack's, per-row constants, and the flag
    raised exactly when a VALID row leaves the to_h5 form (padded rows are only log-encoded)."""
    ops = _ops()
    b, n, c = 2, 37, 13
    tex = _to_h5_texture(b, n, c, 5)
    mask = torch.ones(b, n, dtype=torch.bool)
    mask[1, 30:] = False
    dst = torch.full((b * n,), -1, dtype=torch.int32)
    dst[mask.reshape(-1)] = torch.arange(int(mask.sum()), dtype=torch.int32)
    dst = dst.to(dev)
    t_valid = int(mask.sum())

    def scan(t):
        t = t.clone().to(dev)
        coef = torch.full((t_valid, 16), -7.0, device=dev)
        flag = torch.full((1,), 5, dtype=torch.int32, device=dev)
        ops.texture_scan(t, log_ch, dst, coef, flag)
        return t.cpu(), coef.cpu(), int(flag.item())

    got, coef, flag = scan(tex)
    ref = tex.clone().to(dev)
    ops.texture_pack(ref, log_ch, dst, torch.empty(t_valid, c * 1024, dtype=torch.bfloat16, device=dev))
    assert flag == 0
    assert torch.equal(got, ref.cpu())  # same in-place encode, bit for bit
    exp = got[..., 0, 0].reshape(b * n, c)[mask.reshape(-1)]
    assert torch.equal(coef[:, :c], exp)
    assert torch.all(coef[:, c:] == -7.0)
    bad = tex.clone()
    bad[1, 4, 11, 31, 2] = 0.5  # outside the mask (31 + 2 > 32), valid row
    assert scan(bad)[2] == 1
    bad = tex.clone()
    bad[0, 7, 3, 31, 1] += 0.5  # inside the mask (31 + 1 <= 32), valid row
    assert scan(bad)[2] == 1
    pad_only = tex.clone()
    pad_only[1, 33, 0, 3, 3] += 1.0  # padded row: not checked
    assert scan(pad_only)[2] == 0
    nan = tex.clone()
    nan[0, 0, 5, 0, 0] = float("nan")
    assert scan(nan)[2] == 1


def test_texture_linear_and_gates():
    """rf_texture_linear == bias + coef @ wsum when the flag is 0 and a no-op otherwise; rf_gemm_bf16_if and
    rf_texture_pack_if run only when the flag is set."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(3)
    rows, c, d = 300, 13, 1024
    coef = torch.randn(rows, 16, generator=g).to(dev)
    wsum = torch.randn(c, d, generator=g).to(dev)
    bias = torch.randn(d, generator=g).to(dev)
    out = torch.full((rows, d), 9.0, device=dev)
    flag = torch.ones(1, dtype=torch.int32, device=dev)
    ops.texture_linear(coef, wsum, bias, out, flag)
    assert torch.all(out == 9.0)
    flag.zero_()
    ops.texture_linear(coef, wsum, bias, out, flag)
    ref = bias.double() + coef[:, :c].double() @ wsum.double()
    assert relerr(out, ref) < 1e-6

    a = torch.randn(333, 1024, generator=g).bfloat16().to(dev)
    w = (torch.randn(1024, 1024, generator=g) / 32).bfloat16().to(dev)
    o = torch.full((333, 1024), 9.0, device=dev)
    ops.gemm(a, w, o, bias, ops.EPI_F32, flag=flag)
    tex = _to_h5_texture(1, 20, 13, 1).to(dev)
    dst = torch.arange(20, dtype=torch.int32, device=dev)
    packed = torch.zeros(20, 13 * 1024, dtype=torch.bfloat16, device=dev)
    ops.texture_pack_if(flag, tex, 0, dst, packed)
    torch.cuda.synchronize()
    assert torch.all(o == 9.0) and torch.all(packed == 0)
    flag.fill_(1)
    ops.gemm(a, w, o, bias, ops.EPI_F32, flag=flag)
    assert relerr(o, a.double() @ w.double().t() + bias.double()) < 1e-5
    ops.texture_pack_if(flag, tex, 0, dst, packed)
    assert torch.equal(packed, tex.reshape(20, -1).bfloat16())


def test_texture_embedding_fast_vs_general(monkeypatch):
    """The model's texture embedding on the fast path vs the general pack + GEMM path (bf16 operands)."""
    from renderformer_amd import RenderFormer
    from golden_util import load_case
    cfg, sd, inp, res, z = load_case("tiny_swin")
    m = RenderFormer(cfg, sd).to("cuda")
    mask = inp["mask"].cuda()
    plan = m._plan(mask, 1, res)
    vns = inp["vn"].reshape(mask.shape[0], -1, 9).cuda()
    outs = {}
    for fast in ("1", "0"):
        monkeypatch.setenv("RF_TEX_FAST", fast)
        m._tex_fast = fast == "1"
        outs[fast] = m._embed_triangles(plan, inp["texture"].clone().cuda(), vns, True).cpu()
    assert int(m._w.tex_flag.item()) == 0
    assert relerr(outs["1"], outs["0"]) < 2e-3


def test_attention_schedule_matches_equal_ranges_at_bench_shape():
    """Stage 1 at the bench shape (S = 5,649, 8 heads) on the cost-balanced ranges vs equal tile counts: the
    decompositions differ only in where units are cut — each piece's P = exp2(S - m) is rounded to bf16 on its own
    running-max base — so the outputs agree to bf16-level rounding, and the balanced one is as close to the fp64
    reference as the equal-range one."""
    ops = _ops()
    S, H = 5649, 8
    D = H * 128
    g = torch.Generator(device="cpu").manual_seed(5)
    qkv = torch.randn(S, 3 * D, generator=g).bfloat16().to(dev)
    qs = (qkv[:, :D].float() * ops.Q_LOG2_SCALE).bfloat16()
    probs = [[0, S, 0, S, 0]]
    pt = torch.tensor(probs, dtype=torch.int32, device=dev)
    outs = []
    for sch in (None, ops.attn_schedule(probs, H, dev)):
        out = torch.empty(S, D, device=dev, dtype=torch.bfloat16)
        ops.attention(qs, qkv[:, D:2 * D], qkv[:, 2 * D:], out, pt, S, H, q_prescaled=True, schedule=sch)
        outs.append(out.float())
    assert relerr(outs[1], outs[0]) < 6e-3
    rows = torch.arange(0, S, 97)
    ref = _ref_attn(qs[rows].float().cpu() / ops.Q_LOG2_SCALE, qkv[:, D:2 * D].float().cpu(), qkv[:, 2 * D:].float().cpu(), H)
    e_sched, e_equal = relerr(outs[1][rows].cpu(), ref), relerr(outs[0][rows].cpu(), ref)
    assert e_sched < 6e-3 and e_sched < 1.25 * e_equal, (e_sched, e_equal)


def test_stream_k_epoch_wrap(monkeypatch):
    """stream-K hand-off flags compare against a per-launch epoch that repeats every 2^B launches; on
    each wrap the flag area is re-zeroed on the stream (rf::next_epoch), so a flag left from 2^B launches ago can
    never pass for the current launch's.  With B = 2 (a wrap every 4 launches) repeated attention and stream-K
    GEMM launches with cut units stay correct and raise no device error."""
    monkeypatch.setenv("RF_EPOCH_BITS", "2")
    monkeypatch.setenv("RF_ATTN_GRID", "23")
    ops = _ops()
    H, D = 2, 256
    lens = [700, 129]
    T = sum(lens)
    g = torch.Generator(device="cpu").manual_seed(4)
    qkv = torch.randn(T, 3 * D, generator=g).bfloat16()
    d = qkv.to(dev)
    probs = [[0, 700, 0, 700, 0], [700, 129, 700, 129, 700]]
    pt = torch.tensor(probs, dtype=torch.int32, device=dev)
    a = torch.randn(1000, 1024, generator=g).bfloat16().to(dev)
    w = (torch.randn(1024, 1024, generator=g) / 32).bfloat16().to(dev)
    ref_g = a.double() @ w.double().t()
    monkeypatch.setenv("RF_GEMM_SKPH", "1")
    for it in range(11):
        out = torch.zeros(T, D, device=dev, dtype=torch.bfloat16)
        ops.attention(d[:, :D], d[:, D:2 * D], d[:, 2 * D:], out, pt, 700, H)
        c = torch.empty(1000, 1024, device=dev)
        ops.gemm(a, w, c, None, ops.EPI_F32)
        o = out.float().cpu()
        off = 0
        for n in lens:
            sl = slice(off, off + n)
            ref = _ref_attn(qkv[sl, :D].float(), qkv[sl, D:2 * D].float(), qkv[sl, 2 * D:].float(), H)
            assert relerr(o[sl], ref) < 6e-3, (it, n)
            off += n
        assert relerr(c, ref_g) < 1e-5, it
    torch.cuda.synchronize()
    assert _lib_mod().rf_device_error() == 0


@pytest.mark.parametrize("cin,cout,hh,ww,n_img,n_fin", [(128, 32, 32, 64, 1, 3), (128, 32, 48, 32, 2, 3),
                                                        (64, 16, 16, 32, 1, 4), (256, 24, 32, 32, 1, 3)])
@pytest.mark.parametrize("flags", ["log", "nchw"])
def test_conv_c32_final_head(cin, cout, hh, ww, n_img, n_fin, flags, monkeypatch):
    """output_conv2's kernel (conv3x3_c32_kernel: <= 32 filters, 16 x 32 tiles, fused SiLU -> 1x1 -> ELU -> 10^x - 1
    head) against fp64 on the same fp16 operands, and equal (to fp32 summation order) to the halo2 / engine path it
    replaces (RF_CONV_C32=0)."""
    from renderformer_amd.dpt import FINAL, LOG_DECODE, NCHW_OUT, _Conv, split_planes
    g = torch.Generator(device="cpu").manual_seed(cin + cout + hh)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    b = torch.randn(cout, generator=g) * 0.1
    wf = torch.randn(n_fin, cout, generator=g) / cout ** 0.5
    bf = torch.randn(n_fin, generator=g) * 0.1
    x = torch.randn(n_img, hh, ww, cin, generator=g)
    conv = _Conv(w, b, dev, f16=True)
    xs = split_planes(x.to(dev), conv.cin_pad, f16=True)
    fl = (LOG_DECODE if flags == "log" else NCHW_OUT)
    fin = (wf.to(dev).contiguous(), bf.to(dev).contiguous(), 1e-3)
    got = conv(xs, final=fin, final_flags=fl)
    monkeypatch.setenv("RF_CONV_C32", "0")
    old = _Conv(w, b, dev, f16=True)(xs, final=fin, final_flags=fl)
    xr = x.half().double().permute(0, 3, 1, 2)
    y = F.conv2d(xr, w.half().double(), b.double(), padding=1)
    y = F.silu(y)
    z = torch.einsum("nchw,fc->nfhw", y, wf.double()) + bf.double()[None, :, None, None]
    z = torch.where(z > 0, z, 1e-3 * torch.expm1(z))
    if flags == "log":
        z = (10.0 ** z - 1.0).permute(0, 2, 3, 1)
    assert tuple(got.shape) == tuple(z.shape)
    assert relerr(got.cpu(), z) < 2e-3
    assert relerr(got.cpu(), old.cpu()) < 1e-5
