"""Helpers to load the committed golden fixtures (tests/golden/*.npz)."""
import json
import os

import numpy as np
import torch

from renderformer_amd.config import RenderFormerConfig
from renderformer_amd.scenes import expand_texture
from renderformer_amd.weights import synthetic_state_dict

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["tiny_swin", "tiny_swin_r128", "tiny_full", "tiny_large", "cbox_base"]
# BASELINE.json configs at their own sizes (full depth, make_golden.py): config 2 (large-proxy, cbox, 512^2),
# config 3 (cbox-bunny N=6,209), config 1's shape (v1-base, 256^2), config 5's shape (4 views at 1024^2)
BIG_CASES = ["large_cbox_r512", "large_bunny_r512", "base_cbox_r256", "large_cbox_r1024_v4"]


def reference_hdr(z):
    """(expected HDR, pixel stride): the full image, or for sub-sampled fixtures every stride-th pixel row and
    column (make_golden.HDR_SUB) — compare out[:, :, ::stride, ::stride] against it."""
    if "hdr" in z.files:
        return z["hdr"], 1
    return z["hdr_sub"], int(z["hdr_sub_stride"])


def hdr_shape(z):
    return tuple(int(v) for v in z["hdr_shape"]) if "hdr_shape" in z.files else tuple(z["hdr"].shape)


def load_case(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    cfg = RenderFormerConfig.from_dict(json.loads(str(z["cfg"])))
    sd = synthetic_state_dict(cfg, seed=int(z["weight_seed"]))
    names = [str(n) for n in z["weight_names"]]
    sums = np.array([[float(sd[n].double().sum()), float(sd[n].double().abs().sum())] for n in names])
    if not np.allclose(sums, z["weight_sums"], rtol=1e-9, atol=1e-9):
        raise AssertionError(f"{name}: synthetic weight generator drifted from the fixture")
    inputs = dict(
        triangles=torch.from_numpy(z["triangles"]), vn=torch.from_numpy(z["vn"]),
        texture=torch.from_numpy(expand_texture(z["tex_channels"])), mask=torch.from_numpy(z["mask"]),
        c2w=torch.from_numpy(z["c2w"]), fov=torch.from_numpy(z["fov"]),
    )
    return cfg, sd, inputs, int(z["res"]), z


def rel_l2_ac(a, b):
    """relative L2 of the deviation from the reference image's mean (stricter than rel_l2 on images whose
    values sit on a large constant offset, as random-weight renders do)"""
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    mu = b.mean()
    return float((a - b).norm() / (b - mu).norm().clamp_min(1e-30))


def rel_l2(a, b):
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    return float((a - b).norm() / b.norm().clamp_min(1e-30))
