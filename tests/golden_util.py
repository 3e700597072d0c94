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
# the reference's own example scenes (examples/*.json through the package's converter), large-proxy at 512^2:
# config 4's scenes, incl. the longest triangle sequence (cbox-lucy, S = 11,819)
REAL_CASES = ["real_cbox-lucy_r512", "real_shader-ball_r512", "real_cbox-teapot_r512", "real_init-template_r512",
              "real_room_r512", "real_crystals_r512"]
# cases whose fixture holds production-size intermediate taps (make_golden.PROD_TAPS)
PROD_TAP_CASES = BIG_CASES + ["real_cbox-lucy_r512"]


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
    if "example" in z.files:  # an example scene: regenerate its tensors with the converter and pin them
        from renderformer_amd.examples import inputs_digest, scene_inputs
        a = scene_inputs(str(z["example"]))
        if inputs_digest(a) != str(z["inputs_digest"]):
            raise AssertionError(f"{name}: the converter's output for {z['example']} drifted from the fixture")
        arrays = dict(triangles=a["triangles"][None], vn=a["vn"][None], tex_channels=a["tex_channels"][None],
                      mask=np.ones((1, a["triangles"].shape[0]), dtype=bool), c2w=a["c2w"][None],
                      fov=a["fov"].reshape(1, -1, 1))
    else:
        arrays = {k: z[k] for k in ("triangles", "vn", "tex_channels", "mask", "c2w", "fov")}
    inputs = dict(
        triangles=torch.from_numpy(arrays["triangles"]), vn=torch.from_numpy(arrays["vn"]),
        texture=torch.from_numpy(expand_texture(arrays["tex_channels"])), mask=torch.from_numpy(arrays["mask"]),
        c2w=torch.from_numpy(arrays["c2w"]), fov=torch.from_numpy(arrays["fov"]),
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
