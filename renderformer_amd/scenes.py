"""Synthetic scene generation in the reference's HDF5 tensor format.

Follows SURVEY §8d: triangles uniform in [-0.5, 0.5]^3 (README.md:309),
unit vertex normals, per-triangle constant 13-channel texture patches masked
by ``x + y <= 32`` exactly as ``scene_processor/to_h5.py:42-65`` writes them
(diffuse, specular, roughness, normal, emission), 1-8 emissive triangles at
2,500-5,000 (README.md:310), and look-at cameras (``to_h5.py:10-34``) at
distance 2 with the cbox fov of 37.5 degrees.

Triangle counts of the reference example scenes (counted from their OBJ
files): cbox 5,633; cbox-bunny 6,209; cbox-lucy 11,803;
shader-ball 11,036; init-template 513.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

SCENE_TRIS = {"cbox": 5633, "cbox-bunny": 6209, "cbox-lucy": 11803, "shader-ball": 11036, "init-template": 513}
# triangle counts of all 16 example scenes after conversion (examples/*.json through scene_convert: polygons
# fanned into triangles), in natsort order of the file names (renderformer_amd.examples.example_names)
EXAMPLE_SCENE_TRIS = [5633, 6209, 11803, 9397, 7321, 4527, 3073, 1949, 1418, 5023, 513, 6386, 7141, 11036, 4400, 4575]


def look_at_to_c2w(position, target=(0.0, 0.0, 0.0), up=(0.0, 0.0, 1.0)) -> np.ndarray:
    """Camera-to-world from a look-at triple (restates scene_processor/to_h5.py:10-34)."""
    pos = np.asarray(position, dtype=np.float64)
    fwd = pos - np.asarray(target, dtype=np.float64)
    fwd /= np.linalg.norm(fwd)
    right = np.cross(np.asarray(up, dtype=np.float64), fwd)
    right /= np.linalg.norm(right)
    upv = np.cross(fwd, right)
    upv /= np.linalg.norm(upv)
    w2c = np.eye(4)
    w2c[0, :3], w2c[1, :3], w2c[2, :3] = right, upv, fwd
    t = np.eye(4)
    t[:3, 3] = -pos
    return np.linalg.inv(w2c @ t)


def texture_mask(size: int = 32) -> np.ndarray:
    """to_h5.py:42-45: mask[x, y] = x + y <= size with 'ij' indexing."""
    x, y = np.meshgrid(np.arange(size), np.arange(size), indexing="ij")
    return (x + y) <= size


def expand_texture(channels: np.ndarray, size: int = 32) -> np.ndarray:
    """[..., 13] per-triangle constants -> [..., 13, size, size] masked patches (to_h5.py:63-65), fp16-rounded."""
    tex = np.repeat(np.repeat(channels[..., None, None], size, axis=-2), size, axis=-1)
    tex = tex * texture_mask(size)
    return tex.astype(np.float16).astype(np.float32)


@dataclass
class Scene:
    triangles: np.ndarray   # [N, 3, 3] f32
    vn: np.ndarray          # [N, 3, 3] f32
    tex_channels: np.ndarray  # [N, 13] f32 (fp16-representable)
    c2w: np.ndarray         # [V, 4, 4] f32
    fov: np.ndarray         # [V] f32 degrees


def synthetic_scene(n_tris: int, n_views: int = 1, seed: int = 1, n_lights: Optional[int] = None) -> Scene:
    rng = np.random.default_rng(seed)
    tris = rng.uniform(-0.5, 0.5, size=(n_tris, 3, 3)).astype(np.float32)
    vn = rng.standard_normal((n_tris, 3, 3))
    vn = (vn / np.linalg.norm(vn, axis=-1, keepdims=True)).astype(np.float32)
    ch = np.zeros((n_tris, 13), dtype=np.float64)
    ch[:, 0:3] = rng.uniform(0.0, 0.8, size=(n_tris, 3))
    ch[:, 3:6] = rng.uniform(0.01, 0.5, size=(n_tris, 1))
    ch[:, 6] = rng.uniform(0.01, 1.0, size=n_tris)
    ch[:, 7:10] = (0.5, 0.5, 1.0)
    nl = int(rng.integers(1, 9)) if n_lights is None else n_lights
    lights = rng.choice(n_tris, size=min(nl, n_tris), replace=False)
    ch[lights, 10:13] = rng.uniform(2500.0, 5000.0, size=(len(lights), 1))
    ch = ch.astype(np.float16).astype(np.float32)
    c2w, fov = [], []
    for v in range(n_views):
        ang = 2 * np.pi * v / max(n_views, 1)
        pos = (2.0 * np.sin(ang), -2.0 * np.cos(ang), 0.3 * np.sin(3 * ang))
        c2w.append(look_at_to_c2w(pos))
        fov.append(37.5)
    return Scene(tris, vn, ch, np.stack(c2w).astype(np.float32), np.asarray(fov, dtype=np.float32))


def batch_scenes(scenes, padding_length: Optional[int] = None, expand: bool = True):
    """Collate like batch_infer.py:27-58 (zero padding + mask). Returns a dict of CPU torch tensors."""
    n_max = padding_length or max(s.triangles.shape[0] for s in scenes)
    b = len(scenes)
    v = scenes[0].c2w.shape[0]
    tris = np.zeros((b, n_max, 3, 3), np.float32)
    vn = np.zeros((b, n_max, 3, 3), np.float32)
    ch = np.zeros((b, n_max, 13), np.float32)
    mask = np.zeros((b, n_max), bool)
    for i, s in enumerate(scenes):
        n = s.triangles.shape[0]
        tris[i, :n], vn[i, :n], ch[i, :n], mask[i, :n] = s.triangles, s.vn, s.tex_channels, True
    out = {
        "triangles": torch.from_numpy(tris), "vn": torch.from_numpy(vn), "mask": torch.from_numpy(mask),
        "c2w": torch.from_numpy(np.stack([s.c2w for s in scenes])),
        "fov": torch.from_numpy(np.stack([s.fov for s in scenes]))[..., None],
        "tex_channels": torch.from_numpy(ch),
    }
    if expand:
        out["texture"] = torch.from_numpy(expand_texture(ch))
    return out
