"""MX fp8 (OCP e4m3 + E8M0 block scales) kernels: the device quantiser against the torch float8_e4m3fn
reference of the same rule, and the block-scaled MFMA GEMM (rf_gemm_mx8) against fp64 products of the
dequantised operands (so the test isolates the kernel from the quantisation error)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"


def _ops():
    from renderformer_amd import ops
    return ops


def relerr(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("rows,cols", [(1, 32), (77, 1024), (4096, 4096)])
def test_quant_mx8_matches_reference(rows, cols):
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(rows + cols)
    x = (torch.randn(rows, cols, generator=g) * torch.logspace(-3, 3, cols)[None]).bfloat16()
    x[0, :32] = 0  # an all-zero block
    got = ops.quant_mx8(x.to(dev))
    q_ref, s_ref = ops.mx8_quant_ref(x)
    assert torch.equal(got.s.cpu(), s_ref)
    mism = (got.q.cpu() != q_ref).float().mean().item()
    assert mism == 0.0, f"{mism:.2e} of the e4m3 bytes differ from torch's RNE cast"
    d = ops.mx8_dequant_ref(got.q.cpu(), got.s.cpu())
    assert relerr(d, x.float()) < 0.04  # e4m3: 3 mantissa bits


@pytest.mark.parametrize("m,n,k", [(1, 256, 128), (300, 256, 128), (1000, 512, 1024), (4096, 1024, 4096),
                                   (777, 2048, 384)])
def test_gemm_mx8_vs_fp64(m, n, k):
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(m * 3 + n + k)
    a = torch.randn(m, k, generator=g).bfloat16()
    w = (torch.randn(n, k, generator=g) / math.sqrt(k)).bfloat16()
    aq, wq = ops.quant_mx8(a.to(dev)), ops.quant_mx8(w.to(dev))
    ad = ops.mx8_dequant_ref(aq.q.cpu(), aq.s.cpu()).double()
    wd = ops.mx8_dequant_ref(wq.q.cpu(), wq.s.cpu()).double()
    bias = torch.randn(n, generator=g)
    ref = ad @ wd.t() + bias.double()
    out = torch.empty(m, n, device=dev)
    ops.gemm_mx8(aq, wq, out, bias.to(dev), ops.EPI_F32)
    # (the block-scaled MFMA's internal sum of the fp8 products is not an exact fp32 chain: ~1e-5 measured,
    # three orders below the e4m3 quantisation error)
    assert relerr(out.cpu(), ref) < 1e-4
    acc0 = torch.randn(m, n, generator=g)
    acc = acc0.to(dev)
    ops.gemm_mx8(aq, wq, acc, bias.to(dev), ops.EPI_ADD_F32)
    assert relerr(acc.cpu(), ref + acc0.double()) < 1e-4
    outb = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    ops.gemm_mx8(aq, wq, outb, bias.to(dev), ops.EPI_BF16)
    assert relerr(outb.cpu().float(), ref) < 4e-3
    from renderformer_amd.model import _interleave_swiglu
    wsw = _interleave_swiglu(w[: n // 2], w[n // 2:])
    wsq = ops.quant_mx8(wsw.to(dev))
    wsd = ops.mx8_dequant_ref(wsq.q.cpu(), wsq.s.cpu()).double().view(n // 32, 2, 16, k)
    outs = torch.empty(m, n // 2, device=dev, dtype=torch.bfloat16)
    ops.gemm_mx8(aq, wsq, outs, None, ops.EPI_SWIGLU)
    w1 = wsd[:, 0].reshape(n // 2, k)
    w3 = wsd[:, 1].reshape(n // 2, k)
    refs = F.silu(ad @ w1.t()) * (ad @ w3.t())
    assert relerr(outs.cpu().float(), refs) < 5e-3


def test_gemm_mx8_asymmetric_identity():
    """A = I (exactly representable in e4m3) with an asymmetric W catches a transposed output or a swapped
    scale operand."""
    ops = _ops()
    n = k = 256
    a = torch.eye(k).bfloat16()
    w = (torch.arange(n * k, dtype=torch.float32).view(n, k) % 7 - 3).bfloat16()
    w[5, :] *= 64  # a row whose blocks carry a different scale
    aq, wq = ops.quant_mx8(a.to(dev)), ops.quant_mx8(w.to(dev))
    out = torch.empty(k, n, device=dev)
    ops.gemm_mx8(aq, wq, out, None, ops.EPI_F32)
    assert torch.equal(out.cpu(), w.float().t())
