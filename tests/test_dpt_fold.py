"""The exact DPT rewrite that folds refinenet1's 1x1 out_conv into output_conv1 (renderformer_amd/dpt.py
fold_affine_1x1; reference graph renderformer/layers/dpt.py:147-159, 268-271): checked in float64 on the CPU
against the unfolded composition conv3x3(interpolate(conv1x1(y))) with torch's own ops."""
import torch
import torch.nn.functional as F

from renderformer_amd.dpt import fold_affine_1x1


def _border_bias(b, h, w):
    ry = torch.ones(h, dtype=torch.long)
    rx = torch.ones(w, dtype=torch.long)
    ry[0], ry[-1], rx[0], rx[-1] = 0, 2, 0, 2
    return b[3 * ry[:, None] + rx[None, :]].permute(2, 0, 1)[None]


def test_fold_is_exact_on_upsampled_maps():
    g = torch.Generator().manual_seed(0)
    for ci, cm, co, h, ho, wo in ((5, 6, 4, 7, 17, 17), (8, 8, 3, 4, 8, 8), (3, 5, 2, 6, 13, 9)):
        y = torch.randn(2, ci, h, h, generator=g, dtype=torch.float64)
        w1 = torch.randn(cm, ci, 1, 1, generator=g, dtype=torch.float64)
        b1 = torch.randn(cm, generator=g, dtype=torch.float64)
        w3 = torch.randn(co, cm, 3, 3, generator=g, dtype=torch.float64)
        b3 = torch.randn(co, generator=g, dtype=torch.float64)
        ref = F.conv2d(F.interpolate(F.conv2d(y, w1, b1), (ho, wo), mode="bilinear", align_corners=True), w3, b3,
                       padding=1)
        w, b = fold_affine_1x1(w3, b3, w1, b1)
        assert w.shape == (co, ci, 3, 3) and b.shape == (9, co)
        got = F.conv2d(F.interpolate(y, (ho, wo), mode="bilinear", align_corners=True), w, None, padding=1)
        got = got + _border_bias(b, ho, wo)
        assert float((got - ref).abs().max()) < 1e-11


def test_fold_border_classes_differ_only_by_cut_taps():
    """interior class = b3 + every tap's b1 contribution; a corner drops a row and a column of taps"""
    g = torch.Generator().manual_seed(1)
    w3 = torch.randn(4, 6, 3, 3, generator=g, dtype=torch.float64)
    b3 = torch.randn(4, generator=g, dtype=torch.float64)
    w1 = torch.randn(6, 5, 1, 1, generator=g, dtype=torch.float64)
    b1 = torch.randn(6, generator=g, dtype=torch.float64)
    _, b = fold_affine_1x1(w3, b3, w1, b1)
    tap = torch.einsum("ocyx,c->oyx", w3, b1)
    assert torch.allclose(b[4], b3 + tap.sum((1, 2)))
    assert torch.allclose(b[0], b3 + tap[:, 1:, 1:].sum((1, 2)))
    assert torch.allclose(b[8], b3 + tap[:, :2, :2].sum((1, 2)))
