"""Pin the JSON -> HDF5 converter (renderformer_amd.scene_convert) to the reference's own conversion code.

Run in the build container only (``/root/reference`` does not exist on the GPU box):
``python tests/golden/make_converter_golden.py``.  It imports ``scene_processor`` read-only from
/root/reference.  Its third-party imports are absent here (h5py, trimesh, pymeshlab), so stand-in modules are
put in ``sys.modules`` that only carry data in and out of the reference functions:

* ``trimesh.load`` (to_h5.py:50) returns the object mesh the package's converter built (triangles, per-corner
  normals, face colours = diffuse x 255), i.e. exactly what the reference reads back from its split OBJ files;
* ``h5py.File`` (to_h5.py:87-92) records the datasets ``save_to_h5`` writes instead of writing a file.

So ``save_to_h5`` itself runs: its material packing (channel order, the 0.5/0.5/1 normal channels, emission), the
x + y <= 32 patch mask, the per-patch broadcast, the dtype casts, and ``look_at_to_c2w`` for every camera.  The
unit-sphere normalisation (scene_mesh.py:13-18) runs on a stand-in mesh holding the OBJ's raw vertices.  What the
stand-ins cannot pin is left unpinned and says so in the test: trimesh's rotation matrices, its OBJ round trip
and smooth shading (the geometry the stand-in ``load`` hands over is the package's own).

Writes tests/golden/converter_examples.npz (data only: per example scene, the reference's per-triangle texture
channels, c2w, fov and the normalised vertices of normalised objects).
"""
from __future__ import annotations

import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("RF_REFERENCE", "/root/reference")
sys.path[:0] = [REF, REPO]

from renderformer_amd import scene_convert as sc  # noqa: E402
from renderformer_amd.examples import EXAMPLES_DIR, example_names  # noqa: E402

CAPTURED = {}
MESHES = {}


class _Visual:
    def __init__(self, face_colors):
        self.face_colors = face_colors


class _Mesh:
    """What trimesh.load returns for one split OBJ (to_h5.py:50-55 reads these attributes)."""

    def __init__(self, tris, vn, diffuse):
        n = len(tris)
        self.triangles = tris
        self.faces = np.arange(3 * n).reshape(n, 3)
        self.vertex_normals = vn.reshape(3 * n, 3)
        rgb = np.rint(diffuse * 255.0).astype(np.uint8)
        self.visual = _Visual(np.concatenate([rgb, np.full((n, 1), 255, np.uint8)], axis=1))


class _VertsOnly:
    def __init__(self, v):
        self.vertices = v


class _File:
    def __init__(self, path, mode="r"):
        self.path = path

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def create_dataset(self, name, data=None, **_):
        CAPTURED[name] = np.asarray(data)


def _load(path, process=False, force=None):
    return MESHES[os.path.splitext(os.path.basename(path))[0]]


def install_stubs():
    tm = types.ModuleType("trimesh")
    tm.load = _load
    tm.Trimesh = object
    tm.visual = types.ModuleType("trimesh.visual")
    sys.modules["trimesh"] = tm
    sys.modules["trimesh.visual"] = tm.visual
    h5 = types.ModuleType("h5py")
    h5.File = _File
    sys.modules["h5py"] = h5
    sys.modules["pymeshlab"] = types.ModuleType("pymeshlab")


def main():
    install_stubs()
    from scene_processor.scene_mesh import normalize_to_unit_sphere
    from scene_processor.to_h5 import save_to_h5
    out = {}
    for name in example_names():
        cfg = sc.load_scene_config(os.path.join(EXAMPLES_DIR, name + ".json"))
        if any(o.remesh for o in cfg.objects.values()):
            continue
        MESHES.clear()
        CAPTURED.clear()
        for key, obj in cfg.objects.items():
            tris, vn, ch = sc.object_arrays(obj, EXAMPLES_DIR)
            MESHES[key] = _Mesh(tris, vn, ch[:, :3])
            if obj.transform.normalize:
                v, _ = sc.load_obj(os.path.join(EXAMPLES_DIR, obj.mesh_path))
                out[f"{name}/{key}/normalized"] = normalize_to_unit_sphere(_VertsOnly(v.copy())).vertices
        with tempfile.TemporaryDirectory() as tmp:  # (save_to_h5 makes the output's directory; nothing is written)
            save_to_h5(cfg, os.path.join(tmp, "mesh.obj"), os.path.join(tmp, "out.h5"))
        tex = CAPTURED["texture"]
        out[f"{name}/channels"] = tex[:, :, 0, 0].astype(np.float16)
        out[f"{name}/mask"] = np.any(tex != 0, axis=(0, 1))  # the texels any channel of any triangle uses
        out[f"{name}/c2w"] = CAPTURED["c2w"]
        out[f"{name}/fov"] = CAPTURED["fov"]
        out[f"{name}/tex_nonzero_outside_mask"] = np.array(
            int(np.count_nonzero(tex[:, :, (np.add.outer(np.arange(32), np.arange(32)) > 32)])))
        print(f"{name}: {tex.shape[0]} triangles, {CAPTURED['c2w'].shape[0]} cameras")
    np.savez_compressed(os.path.join(HERE, "converter_examples.npz"), **out)
    print(f"wrote {len(out)} arrays")


if __name__ == "__main__":
    main()
