"""Generate golden fixtures by running the *reference* RenderFormer on CPU fp32.

Run in the build container only (``/root/reference`` does not exist on the GPU
box):  ``python tests/golden/make_golden.py``.  It imports the reference
package read-only from /root/reference with the ``roma`` stand-in in
``tests/golden/shim`` and ``ATTN_IMPL=sdpa`` (flash_attn is absent; the
reference falls back to SDPA itself, attention.py:29-32), loads the
build-defined synthetic weights with ``load_state_dict(strict=True)`` and
writes small ``.npz`` files next to this script:

* inputs in the HDF5 tensor format (per-triangle texture channels; the 32x32
  patches are re-expanded deterministically by ``scenes.expand_texture``),
* the weight seed plus per-tensor checksums (guards generator drift),
* intermediate taps (stage-1 input/output, decoder layer outputs, DPT logits,
  rays, camera-frame triangles) for the small cases, and
* the final HDR output ``[B, V, res, res, 3]``.

Only data is written; no reference source is copied.
"""
from __future__ import annotations

import json
import os
import sys
import time
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("RF_REFERENCE", "/root/reference")

os.environ["ATTN_IMPL"] = "sdpa"
sys.path[:0] = [os.path.join(HERE, "shim"), REF, REPO]
warnings.filterwarnings("ignore")

import torch  # noqa: E402

from renderformer_amd.config import LARGE_PROXY, RenderFormerConfig  # noqa: E402
from renderformer_amd.scenes import batch_scenes, synthetic_scene  # noqa: E402
from renderformer_amd.weights import synthetic_state_dict  # noqa: E402

LARGE = LARGE_PROXY.to_dict()
BASE = {}
TINY = dict(latent_dim=256, num_layers=2, num_heads=2, dim_feedforward=512, view_transformer_latent_dim=256,
            view_transformer_ffn_hidden_dim=512, view_transformer_n_heads=2, view_transformer_n_layers=4,
            dpt_features=32, dpt_out_channels=[16, 32, 64, 128])

CASES = {
    # name: (config overrides, [n_tris per scene], padding_length, n_views, res, weight seed, scene seed, taps)
    "tiny_swin": (dict(TINY, view_transformer_use_swin_attn=True), [61, 45], 64, 2, 64, 0, 11, True),
    "tiny_swin_r128": (dict(TINY, view_transformer_use_swin_attn=True), [70], None, 1, 128, 1, 12, True),
    "tiny_full": (dict(TINY, view_transformer_use_swin_attn=False), [53], None, 2, 64, 2, 13, True),
    "tiny_large": (dict(latent_dim=1024, num_layers=1, num_heads=8, dim_feedforward=4096,
                        view_transformer_latent_dim=1024, view_transformer_ffn_hidden_dim=4096,
                        view_transformer_n_heads=8, view_transformer_n_layers=4,
                        view_transformer_use_swin_attn=True, dpt_features=256,
                        dpt_out_channels=[128, 256, 512, 1024]), [100], None, 1, 64, 3, 14, False),
    "cbox_base": (dict(num_layers=2, view_transformer_n_layers=4, view_transformer_use_swin_attn=True),
                  [5633], None, 1, 64, 4, 15, False),
    # BASELINE.json configs at their own sizes (full depth).  Weight seed 0 and scene seed 1 are bench.py's
    # headline workload, so bench's frame can be checked against this fixture too.
    "large_cbox_r512": (LARGE, [5633], None, 1, 512, 0, 1, False),       # config 2
    "large_bunny_r512": (LARGE, [6209], None, 1, 512, 0, 2, False),      # config 3 (cbox-bunny N)
    "base_cbox_r256": (BASE, [5633], None, 1, 256, 0, 3, False),         # config 1 shape (v1-base, full depth)
    "large_cbox_r1024_v4": (LARGE, [5633], None, 4, 1024, 0, 4, False),  # config 5 shape, 4 views of 1 scene
}
# The reference's own example scenes (examples/*.json, converted by renderformer_amd.examples: the fixture
# records the digest of the converted tensors instead of the tensors): config 4's scenes, incl. the longest
# triangle sequence (cbox-lucy, N = 11,803 -> S = 11,819).  name: (example, config, res, weight seed, unused)
REAL_CASES = {
    "real_cbox-lucy_r512": ("cbox-lucy", LARGE, 512, 0, True),
    "real_shader-ball_r512": ("shader-ball", LARGE, 512, 0, False),
    "real_cbox-teapot_r512": ("cbox-teapot", LARGE, 512, 0, False),
    "real_init-template_r512": ("init-template", LARGE, 512, 0, False),
    "real_room_r512": ("room", LARGE, 512, 0, False),
    "real_crystals_r512": ("crystals", LARGE, 512, 0, False),
}
# 1024^2 x 4 views is 50 MB of fp32 HDR: such fixtures keep every SUB-th pixel row and column (plus the
# full-image sum and sum of squares), the GPU test compares the same sample
HDR_SUB = {"large_cbox_r1024_v4": 4, **{n: 2 for n in REAL_CASES}}
# production-size intermediate taps (the big cases): a fixed row sample of the stage-1 output (the 16 register
# rows + seeded triangle rows), of every decoder layer's output (seeded ray-token rows of the first views) and
# the pre-ELU DPT logits every DPT_SUB-th pixel
PROD_TAPS = {"large_cbox_r512", "large_bunny_r512", "base_cbox_r256", "large_cbox_r1024_v4", "real_cbox-lucy_r512"}
N_ENC_ROWS, N_DEC_ROWS, N_DEC_VIEWS = 128, 16, 2
DPT_SUB = {256: 2, 512: 4, 1024: 8}


def weight_checksums(sd):
    names = sorted(sd)
    return names, np.array([[float(sd[n].double().sum()), float(sd[n].double().abs().sum())] for n in names])


def tap_rows(name, S, R, V):
    """The fixed row samples of a production-size case: stage-1 rows (16 register rows + seeded triangle rows),
    decoder ray-token rows (the same rows in each recorded view), the recorded views."""
    g = np.random.default_rng(sum(map(ord, name)))
    enc = np.concatenate([np.arange(16), np.sort(g.choice(np.arange(16, S), N_ENC_ROWS - 16, replace=False))])
    dec = np.sort(g.choice(R, N_DEC_ROWS, replace=False))
    return enc.astype(np.int64), dec.astype(np.int64), np.arange(min(V, N_DEC_VIEWS), dtype=np.int64)


def real_batch(example):
    """One example scene (examples/<example>.json through this package's converter) as a batch of one."""
    from renderformer_amd.examples import inputs_digest, scene_inputs
    from renderformer_amd.scenes import expand_texture
    a = scene_inputs(example)
    b = {k: torch.from_numpy(v)[None] for k, v in a.items() if k != "fov"}
    b["fov"] = torch.from_numpy(a["fov"]).reshape(1, -1, 1)
    b["mask"] = torch.ones(1, a["triangles"].shape[0], dtype=torch.bool)
    b["texture"] = torch.from_numpy(expand_texture(a["tex_channels"]))[None]
    return b, inputs_digest(a)


def run_case(name, over, ntris, pad, nv, res, wseed, sseed, taps, example=None):
    from renderformer.models.config import RenderFormerConfig as RefConfig
    from renderformer.models.renderformer import RenderFormer as RefModel
    from renderformer.pipelines.rendering_pipeline import RenderFormerRenderingPipeline as RefPipeline

    cfg = RenderFormerConfig(**over)
    sd = synthetic_state_dict(cfg, seed=wseed)
    model = RefModel(RefConfig(**over))
    model.load_state_dict(sd, strict=True)
    model.eval()
    pipe = RefPipeline(model)

    digest = None
    if example is not None:
        batch, digest = real_batch(example)
        nv = int(batch["c2w"].shape[1])
    else:
        scenes = [synthetic_scene(n, nv, seed=sseed + i) for i, n in enumerate(ntris)]
        batch = batch_scenes(scenes, padding_length=pad)
    tex = batch["texture"].clone()
    t0 = time.time()

    got = {}
    hooks = []
    prod = name in PROD_TAPS
    S = int(batch["mask"][0].sum()) + cfg.num_register_tokens
    R = (res // cfg.patch_size) ** 2
    if prod:
        enc_idx, dec_idx, dec_views = tap_rows(name, S, R, nv)
        got["enc_row_idx"] = torch.from_numpy(enc_idx)
        got["dec_row_idx"] = torch.from_numpy(dec_idx)
        got["dec_views"] = torch.from_numpy(dec_views)
        hooks.append(model.transformer.register_forward_hook(
            lambda m, a, o: got.__setitem__("enc_rows", o[0, enc_idx].clone())))
        dec_rows = []
        for i, layer in enumerate(model.view_transformer.transformer.layers):
            hooks.append(layer.register_forward_hook(
                lambda m, a, o: dec_rows.append(o[dec_views][:, dec_idx].clone())))
        sub = DPT_SUB[res]
        hooks.append(model.view_transformer.out_dpt.register_forward_hook(
            lambda m, a, o: got.__setitem__("dpt_sub", o[:, :, ::sub, ::sub].clone())))
    if not taps:  # size-independent signature of stage 1 at production sequence length
        hooks.append(model.transformer.register_forward_hook(
            lambda m, a, o: got.__setitem__("enc_rownorm", o.norm(dim=-1).clone())))
    if taps:
        hooks.append(model.transformer.register_forward_pre_hook(lambda m, a: got.__setitem__("seq0", a[0].clone())))
        hooks.append(model.transformer.register_forward_hook(lambda m, a, o: got.__setitem__("enc_out", o.clone())))
        for i, layer in enumerate(model.view_transformer.transformer.layers):
            hooks.append(layer.register_forward_hook(
                lambda m, a, o, i=i: got.__setitem__(f"dec{i}", o.clone())))
        hooks.append(model.view_transformer.out_dpt.register_forward_hook(
            lambda m, a, o: got.__setitem__("dpt", o.clone())))
    with torch.no_grad():
        out = pipe.render(batch["triangles"], tex, batch["mask"], batch["vn"], batch["c2w"], batch["fov"],
                          resolution=res, torch_dtype=torch.float32)
    for h in hooks:
        h.remove()
    if prod:
        got["dec_rows"] = torch.stack(dec_rows)  # [layers, views, rows, D]
        got["dpt_sub_stride"] = torch.tensor(DPT_SUB[res])

    names, sums = weight_checksums(sd)
    rec = dict(
        cfg=json.dumps(cfg.to_dict()), weight_seed=np.int64(wseed), weight_names=np.array(names),
        weight_sums=sums, res=np.int64(res), texture_after_ch10=tex[:, :, 10, 0, 0].numpy(),
    )
    if example is None:
        rec.update(triangles=batch["triangles"].numpy(), vn=batch["vn"].numpy(),
                   tex_channels=batch["tex_channels"].numpy(), mask=batch["mask"].numpy(), c2w=batch["c2w"].numpy(),
                   fov=batch["fov"].numpy())
    else:  # the converted example: its tensors are regenerated by the tests and checked against this digest
        rec.update(example=np.array(example), inputs_digest=np.array(digest))
    sub = HDR_SUB.get(name)
    if sub:
        o64 = out.double()
        rec.update(hdr_sub=out[:, :, ::sub, ::sub].numpy().astype(np.float32), hdr_sub_stride=np.int64(sub),
                   hdr_shape=np.array(out.shape), hdr_sum=np.float64(o64.sum()), hdr_sumsq=np.float64((o64 ** 2).sum()))
    else:
        rec["hdr"] = out.numpy().astype(np.float32)
    if nv >= 2:  # how far apart two views of the scene are (the tests' discrimination guard)
        a, b = out[0, 1].double(), out[0, 0].double()
        rec["view01_rel_l2"] = np.float64((a - b).norm() / b.norm())
        rec["view01_rel_l2_ac"] = np.float64((a - b).norm() / (b - b.mean()).norm())
    for k, v in got.items():
        if k.endswith("_idx") or k in ("dec_views", "dpt_sub_stride"):
            rec[k] = v.numpy().astype(np.int64)
            continue
        key = k if k == "enc_rownorm" else "tap_" + k
        rec[key] = v.numpy().astype(np.float32)
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **rec)
    print(f"{name}: {time.time() - t0:.1f} s, hdr {tuple(out.shape)} range [{out.min():.3g}, {out.max():.3g}] -> {os.path.getsize(path)/1e6:.2f} MB")


def op_level():
    """Op-level known answers: triangle RoPE tables, NeRF encoding, Swin mask, rays, camera transform."""
    from renderformer.encodings.nerf_encoding import NeRFEncoding
    from renderformer.encodings.rope import TriangleRotaryEmbedding, freqs_to_cos_sin
    from renderformer.layers.attention import get_swin_attn_mask
    from renderformer.utils.ray_generator import RayGenerator
    from renderformer.utils.transform import trans_to_cam_coord

    g = torch.Generator().manual_seed(5)
    pos = torch.rand(2, 37, 9, generator=g) * 2 - 1
    rope = TriangleRotaryEmbedding(dim=12)
    cos, sin = freqs_to_cos_sin(rope.get_triangle_freqs(pos), head_dim=128)
    vn = torch.randn(3, 5, 9, generator=g)
    nerf = NeRFEncoding(in_dim=9, num_frequencies=6, include_input=True)(vn)
    m16 = get_swin_attn_mask(16, 16, 8, 4, "cpu")
    m8 = get_swin_attn_mask(8, 8, 8, 4, "cpu")
    c2w = torch.randn(2, 4, 4, generator=g)
    c2w[:, 3] = torch.tensor([0.0, 0, 0, 1])
    q, _ = torch.linalg.qr(torch.randn(2, 3, 3, generator=g))
    c2w[:, :3, :3] = q
    fov = torch.full((2, 1), 0.6)
    ro, rd = RayGenerator()(c2w, fov, 32)
    tris = torch.randn(2, 7, 3, 3, generator=g)
    tcam, _, _ = trans_to_cam_coord(c2w, tris)
    np.savez_compressed(os.path.join(HERE, "ops.npz"), rope_pos=pos.numpy(), rope_freqs=rope.freqs.detach().numpy(),
                        rope_cos=cos.numpy(), rope_sin=sin.numpy(), nerf_in=vn.numpy(), nerf_out=nerf.numpy(),
                        swin_mask16=m16.numpy(), swin_mask8=m8.numpy(), c2w=c2w.numpy(), fov=fov.numpy(),
                        rays_o=ro.numpy(), rays_d=rd.numpy(), tris=tris.numpy(), tris_cam=tcam.numpy())
    print("ops.npz written")


if __name__ == "__main__":
    torch.set_num_threads(os.cpu_count() or 8)
    only = sys.argv[1:]
    if not only:
        op_level()
    for name, args in CASES.items():
        if not only or name in only:
            run_case(name, *args)
    for name, (example, over, res, wseed, taps) in REAL_CASES.items():
        if not only or name in only:
            run_case(name, over, None, None, 1, res, wseed, 0, False, example=example)
