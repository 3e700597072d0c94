"""Scene JSON -> HDF5 conversion (restates scene_processor/{convert_scene,scene_mesh,to_h5,scene_config}.py).

The reference converts a scene description (examples/*.json, schema scene_config.py:1-81) in two passes:
``generate_scene_mesh`` (scene_mesh.py:21-93) loads every object's OBJ with trimesh, normalises / rotates /
scales / translates it, smooth-shades it (``trimesh.graph.smooth_shade``, 30 degrees) or splits it flat,
assigns diffuse colours and exports one OBJ per object; ``save_to_h5`` (to_h5.py:37-92) reloads those OBJs and
writes ``triangles[N,3,3] f32``, ``vn[N,3,3] f32``, ``texture[N,13,32,32] f16`` (per-triangle constants x the
``i + j <= 32`` patch mask), ``c2w[V,4,4] f32`` (look-at, to_h5.py:10-34) and ``fov[V] f32``, gzip level 9.

This module does the same in numpy with no trimesh/h5py/dacite (none is installed here):

* OBJ parsing (``v``/``f`` records, polygons fanned, negative indices), ``process=False`` semantics: vertices
  are kept as written, nothing is merged.
* Transforms exactly as scene_mesh.py:41-55: unit-sphere normalisation (:13-18), rotations about x, y, z in that
  order, per-axis scale, translation.
* Smooth shading: faces are grouped by edge adjacency across dihedral angles below 30 degrees, with
  trimesh's large-facet rule (coplanar facets over 1/10 of the mesh area are shaded alone, ``smooth_groups``);
  every group gets its own copy of its vertices and angle-weighted vertex normals.  This restates what
  trimesh.graph.smooth_shade does, but trimesh is third-party and absent, so the grouping details (facet
  coplanarity test, group order) and the normal weighting are PARITY UNPINNED
  (for the planar-walled example scenes such as cbox every group is planar and the normals are the plane
  normals under any weighting).  Flat shading: per-face vertices, normals = face normals.
* The OBJ round trip of the reference (export at 8 decimals, reload) is reproduced by rounding vertices and
  normals to 8 decimals before the float32 cast.
* Diffuse colour through uint8 vertex colours ((d * 255).clip(0, 255).astype(int) / 255, scene_mesh.py:87-90),
  or seeded random colours per shading group / per triangle (scene_mesh.py:63-84, np.random.seed + randint in
  component order; component order parity unpinned).
* ``remesh`` needs pymeshlab (scene_processor/remesh.py) and is rejected.
"""
from __future__ import annotations

import dataclasses
import json
import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from .h5io import write_scene
from .scenes import look_at_to_c2w, texture_mask

SMOOTH_ANGLE = math.radians(30.0)  # scene_mesh.py:58


# ------------------------------------------------------------------------------------------- schema
@dataclass
class TransformConfig:
    translation: List[float]
    rotation: List[float]
    scale: List[float]
    normalize: bool = True


@dataclass
class MaterialConfig:
    diffuse: List[float]
    specular: List[float]
    roughness: float
    emissive: List[float]
    smooth_shading: bool
    rand_tri_diffuse_seed: Optional[int] = None
    random_diffuse_max: float = 1.0
    random_diffuse_type: str = "per-shading-group"


@dataclass
class ObjectConfig:
    mesh_path: str
    material: MaterialConfig
    transform: TransformConfig
    remesh: bool = False
    remesh_target_face_num: int = 2048


@dataclass
class CameraConfig:
    position: List[float]
    look_at: List[float]
    up: List[float]
    fov: float


@dataclass
class SceneConfig:
    scene_name: str
    version: str
    objects: Dict[str, ObjectConfig]
    cameras: List[CameraConfig]


_NESTED = {("ObjectConfig", "material"): MaterialConfig, ("ObjectConfig", "transform"): TransformConfig}


def _check_type(cls_name, name, value, tp):
    ok = True
    if tp in (float,):
        ok = isinstance(value, (int, float)) and not isinstance(value, bool)
    elif tp is int:
        ok = isinstance(value, int) and not isinstance(value, bool)
    elif tp is bool:
        ok = isinstance(value, bool)
    elif tp is str:
        ok = isinstance(value, str)
    elif tp == List[float]:
        ok = isinstance(value, list) and all(isinstance(v, (int, float)) and not isinstance(v, bool) for v in value)
    elif tp == Optional[int]:
        ok = value is None or (isinstance(value, int) and not isinstance(value, bool))
    if not ok:
        raise TypeError(f"{cls_name}.{name}: wrong value type {type(value).__name__}")


def _from_dict(cls, data):
    """dacite.from_dict(check_types=True, strict=True) for this schema: unknown keys and type mismatches raise."""
    if not isinstance(data, dict):
        raise TypeError(f"{cls.__name__}: expected an object")
    fields = {f.name: f for f in dataclasses.fields(cls)}
    extra = set(data) - set(fields)
    if extra:
        raise ValueError(f"{cls.__name__}: unexpected field(s) {sorted(extra)}")
    kw = {}
    for name, f in fields.items():
        if name not in data:
            if f.default is dataclasses.MISSING and f.default_factory is dataclasses.MISSING:
                raise ValueError(f"{cls.__name__}: missing field {name!r}")
            continue
        v = data[name]
        sub = _NESTED.get((cls.__name__, name))
        if sub is not None:
            v = _from_dict(sub, v)
        elif cls is SceneConfig and name == "objects":
            if not isinstance(v, dict):
                raise TypeError("SceneConfig.objects: expected an object")
            v = {k: _from_dict(ObjectConfig, o) for k, o in v.items()}
        elif cls is SceneConfig and name == "cameras":
            if not isinstance(v, list):
                raise TypeError("SceneConfig.cameras: expected a list")
            v = [_from_dict(CameraConfig, c) for c in v]
        else:
            _check_type(cls.__name__, name, v, f.type if not isinstance(f.type, str) else eval(f.type))
        if cls is MaterialConfig and name == "random_diffuse_type" and v not in ("per-triangle", "per-shading-group"):
            raise ValueError(f"MaterialConfig.random_diffuse_type: {v!r}")
        kw[name] = v
    return cls(**kw)


def load_scene_config(path: str) -> SceneConfig:
    with open(path) as f:
        return _from_dict(SceneConfig, json.load(f))


# ------------------------------------------------------------------------------------------- meshes
def load_obj(path: str):
    """Vertices [V,3] f64 and triangle faces [F,3] (0-based) of an OBJ; polygons are fanned (0,i,i+1)."""
    verts, faces = [], []
    with open(path) as f:
        for line in f:
            if line.startswith("v "):
                verts.append([float(t) for t in line.split()[1:4]])
            elif line.startswith("f "):
                idx = []
                for tok in line.split()[1:]:
                    i = int(tok.split("/")[0])
                    idx.append(i - 1 if i > 0 else len(verts) + i)
                for j in range(1, len(idx) - 1):
                    faces.append([idx[0], idx[j], idx[j + 1]])
    return np.asarray(verts, dtype=np.float64).reshape(-1, 3), np.asarray(faces, dtype=np.int64).reshape(-1, 3)


def _rotation(axis: int, deg: float) -> np.ndarray:
    c, s = math.cos(math.radians(deg)), math.sin(math.radians(deg))
    i, j = [(1, 2), (2, 0), (0, 1)][axis]
    r = np.eye(3)
    r[i, i], r[i, j], r[j, i], r[j, j] = c, -s, s, c
    return r


def transform_vertices(v: np.ndarray, t: TransformConfig) -> np.ndarray:
    """scene_mesh.py:31-55: [normalise to unit sphere], rotate x then y then z, scale, translate."""
    v = v.copy()
    if t.normalize:  # normalize_to_unit_sphere (scene_mesh.py:13-18)
        v = v - v.mean(axis=0)
        v = v / (np.linalg.norm(v, ord=2, axis=-1).max() * 2.0)
    for axis, ang in enumerate(t.rotation):
        v = v @ _rotation(axis, ang).T
    v = v * np.asarray(t.scale, dtype=np.float64)
    return v + np.asarray(t.translation, dtype=np.float64)


def _face_normals(tris: np.ndarray) -> np.ndarray:
    n = np.cross(tris[:, 1] - tris[:, 0], tris[:, 2] - tris[:, 0])
    ln = np.linalg.norm(n, axis=1, keepdims=True)
    return np.where(ln > 0, n / np.where(ln > 0, ln, 1), 0.0)


def _face_angles(tris: np.ndarray) -> np.ndarray:
    out = np.zeros(tris.shape[:2])
    for k in range(3):
        a = tris[:, (k + 1) % 3] - tris[:, k]
        b = tris[:, (k + 2) % 3] - tris[:, k]
        cosang = (a * b).sum(1) / np.maximum(np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1), 1e-300)
        out[:, k] = np.arccos(np.clip(cosang, -1.0, 1.0))
    return out


# trimesh.graph.facets declares two adjacent faces coplanar when (face_adjacency_radius / span)^2 exceeds
# tol.facet_threshold = 5000; with radius = span / (2 sin(theta / 2)) that is a dihedral angle below
# 2 asin(1 / (2 sqrt(5000))) = 0.81 degrees (restated from trimesh's published source, which is not installed
# here: PARITY UNPINNED, like the rest of the smooth-shading restatement)
FACET_ANGLE = 2.0 * math.asin(1.0 / (2.0 * math.sqrt(5000.0)))
FACET_MINAREA = 10.0  # smooth_shade's default: facets larger than mesh.area / 10 are shaded on their own


def _components(n: int, pairs, keep=None) -> List[List[int]]:
    """Connected components of faces 0..n-1 over the given adjacency pairs (union-find), ordered by their first
    face; with ``keep`` only those faces take part."""
    parent = np.arange(n)

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    for a, b in pairs:
        ra, rb = find(a), find(b)
        if ra != rb:
            parent[max(ra, rb)] = min(ra, rb)
    order, seen = [], {}
    for fi in range(n):
        if keep is not None and not keep[fi]:
            continue
        r = find(fi)
        if r not in seen:
            seen[r] = len(order)
            order.append([])
        order[seen[r]].append(fi)
    return order


def smooth_groups(v: np.ndarray, f: np.ndarray, angle: float = SMOOTH_ANGLE,
                  facet_minarea: Optional[float] = FACET_MINAREA) -> List[np.ndarray]:
    """Shading groups of trimesh.graph.smooth_shade(mesh, angle, facet_minarea) (scene_mesh.py:58):
    faces joined through shared edges whose dihedral angle is below `angle`, except that every facet (a
    connected set of >= 2 coplanar faces) with more than 1/facet_minarea of the mesh's area is cut out of that
    adjacency and becomes a group of its own, so large flat regions keep their plane normals and do not bend
    their neighbours' normals.  Order: the smoothed components, then the large facets, then faces left alone.
    Group order only orders triangles in the output (the renderer is invariant to it); the seeded random
    colours follow it."""
    tris = v[f]
    fn = _face_normals(tris)
    edges = {}
    for fi, (a, b, c) in enumerate(f):
        for e in ((a, b), (b, c), (c, a)):
            edges.setdefault((min(e), max(e)), []).append(fi)
    adj, dih = [], []
    for fs in edges.values():
        for i in range(len(fs)):
            for j in range(i + 1, len(fs)):
                a, b = fs[i], fs[j]
                adj.append((a, b))
                dih.append(math.acos(max(-1.0, min(1.0, float(fn[a] @ fn[b])))))
    n = len(f)
    smooth = [p for p, d in zip(adj, dih) if d < angle]
    facets = []
    if facet_minarea is not None and smooth:
        area = 0.5 * np.linalg.norm(np.cross(tris[:, 1] - tris[:, 0], tris[:, 2] - tris[:, 0]), axis=-1)
        flat = [p for p, d in zip(adj, dih) if d < FACET_ANGLE]
        cand = [g for g in _components(n, flat) if len(g) >= 2]
        facets = [g for g in cand if area[g].sum() > area.sum() / facet_minarea]
    if not facets:
        return [np.asarray(g, dtype=np.int64) for g in _components(n, smooth)]
    free = np.ones(n, dtype=bool)
    for g in facets:
        free[g] = False
    smooth = [(a, b) for a, b in smooth if free[a] and free[b]]
    in_pair = np.zeros(n, dtype=bool)
    for a, b in smooth:
        in_pair[a] = in_pair[b] = True
    groups = _components(n, smooth, keep=in_pair)  # connected_components(min_len=2) over the remaining pairs
    groups += facets
    covered = np.zeros(n, dtype=bool)
    for g in groups:
        covered[g] = True
    groups += [[int(i)] for i in np.flatnonzero(~covered)]  # loose faces, one group each
    return [np.asarray(g, dtype=np.int64) for g in groups]


def vertex_normals(v: np.ndarray, f: np.ndarray) -> np.ndarray:
    """Angle-weighted vertex normals (face normal x corner angle, summed, normalised)."""
    tris = v[f]
    fn = _face_normals(tris)
    w = _face_angles(tris)
    acc = np.zeros_like(v)
    for k in range(3):
        np.add.at(acc, f[:, k], fn * w[:, k:k + 1])
    ln = np.linalg.norm(acc, axis=1, keepdims=True)
    return np.where(ln > 0, acc / np.where(ln > 0, ln, 1), 0.0)


def shade(v: np.ndarray, f: np.ndarray, smooth: bool):
    """(triangles [F,3,3], per-corner normals [F,3,3], group id per face) after smooth or flat shading."""
    if not smooth:
        tris = v[f]
        fn = _face_normals(tris)
        return tris, np.repeat(fn[:, None], 3, axis=1), np.arange(len(f))
    tris, vns, gid = [], [], []
    for g, faces in enumerate(smooth_groups(v, f, facet_minarea=FACET_MINAREA)):
        used, local = np.unique(f[faces], return_inverse=True)
        lf = local.reshape(-1, 3)
        lv = v[used]
        tris.append(lv[lf])
        vns.append(vertex_normals(lv, lf)[lf])
        gid.append(np.full(len(faces), g))
    return np.concatenate(tris), np.concatenate(vns), np.concatenate(gid)


def object_arrays(obj: ObjectConfig, scene_dir: str):
    """(triangles [n,3,3] f64, vn [n,3,3] f64, channels [n,13] f64) of one object."""
    if obj.remesh:
        raise NotImplementedError("remesh needs pymeshlab (scene_processor/remesh.py), which is not available")
    v, f = load_obj(os.path.join(scene_dir, obj.mesh_path))
    v = transform_vertices(v, obj.transform)
    tris, vn, gid = shade(v, f, obj.material.smooth_shading)
    tris = np.round(tris, 8)  # the reference's OBJ export / reload (8 decimals)
    vn = np.round(vn, 8)
    n = len(tris)
    m = obj.material
    if m.rand_tri_diffuse_seed is not None:
        np.random.seed(m.rand_tri_diffuse_seed)
        comp = np.arange(n) if m.random_diffuse_type == "per-triangle" else gid
        colors = np.zeros((n, 3))
        for c in range(int(comp.max()) + 1 if n else 0):
            sel = comp == c
            colors[sel] = np.random.randint(0, math.ceil(256 * m.random_diffuse_max), (1, 3))
        diffuse = colors / 255.0
    else:
        diffuse = np.repeat((np.array(m.diffuse) * 255.0).clip(0, 255).astype(int)[None] / 255.0, n, axis=0)
    ch = np.concatenate([
        diffuse,
        np.repeat(np.asarray(m.specular, dtype=np.float64)[None], n, axis=0),
        np.full((n, 1), float(m.roughness)),
        np.repeat(np.array([[0.5, 0.5, 1.0]]), n, axis=0),
        np.repeat(np.asarray(m.emissive, dtype=np.float64)[None], n, axis=0),
    ], axis=1)
    return tris, vn, ch


def scene_arrays(cfg: SceneConfig, scene_dir: str, size: int = 32):
    """The five HDF5 datasets of to_h5.py:87-92 (before their dtype casts)."""
    tris, vns, chs = [], [], []
    for obj in cfg.objects.values():
        t, n, c = object_arrays(obj, scene_dir)
        tris.append(t)
        vns.append(n)
        chs.append(c)
    tris, vns, chs = np.concatenate(tris), np.concatenate(vns), np.concatenate(chs)
    tex = np.repeat(np.repeat(chs[..., None], size, axis=-1)[..., None], size, axis=-1)
    tex[:, :, ~texture_mask(size)] = 0.0
    c2w = np.stack([look_at_to_c2w(c.position, c.look_at, c.up) for c in cfg.cameras])
    fov = np.array([c.fov for c in cfg.cameras])
    return {"triangles": tris, "vn": vns, "texture": tex, "c2w": c2w, "fov": fov}


def convert_scene(config_path: str, output_h5_path: Optional[str] = None, compression_level: int = 9) -> str:
    """convert_scene.py:11-45 without the intermediate mesh files: JSON -> HDF5 (returns the written path)."""
    cfg = load_scene_config(config_path)
    out = output_h5_path or os.path.splitext(config_path)[0] + ".h5"
    arr = scene_arrays(cfg, os.path.dirname(os.path.abspath(config_path)))
    if os.path.dirname(out):
        os.makedirs(os.path.dirname(out), exist_ok=True)
    write_scene(out, arr["triangles"], arr["vn"], arr["texture"], arr["c2w"], arr["fov"],
                compression_level=compression_level)
    return out
