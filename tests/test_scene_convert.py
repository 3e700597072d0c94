"""JSON -> HDF5 scene conversion (renderformer_amd.scene_convert, restating scene_processor/*.py).

Fixture: the reference's own examples/cbox.json and the OBJ files it lists (examples/ at the repository root, data
copied from the reference's examples/).  Pinned: dataset names / shapes / dtypes (to_h5.py:87-92), the
texture patch layout (constant x {i + j <= 32}, to_h5.py:41-66), the look-at camera (to_h5.py:10-34),
the transforms (scene_mesh.py:31-55) and the uint8 diffuse round trip (:87-90).  The smooth-shading normals
come from trimesh in the reference (absent here): parity unpinned, checked only for the planar case where any
weighting gives the plane normal.
"""
import json
import math
import os

import numpy as np
import pytest
import torch

from renderformer_amd import h5io
from renderformer_amd import scene_convert as sc
from renderformer_amd.scenes import texture_mask

HERE = os.path.dirname(os.path.abspath(__file__))
CBOX = os.path.join(os.path.dirname(HERE), "examples", "cbox.json")


def test_cbox_converts_to_reference_format(tmp_path):
    out = sc.convert_scene(CBOX, str(tmp_path / "cbox.h5"))
    with h5io.File(out) as f:
        tri, vn, tex = np.array(f["triangles"]), np.array(f["vn"]), np.array(f["texture"])
        c2w, fov = np.array(f["c2w"]), np.array(f["fov"])
    n = 4 * 128 + 2 * 2560 + 1  # cbox = 5,633 triangles
    assert tri.shape == (n, 3, 3) and tri.dtype == np.float32 and vn.shape == (n, 3, 3) and vn.dtype == np.float32
    assert tex.shape == (n, 13, 32, 32) and tex.dtype == np.float16
    assert c2w.shape == (1, 4, 4) and fov.tolist() == [37.5]
    # texture: every channel constant inside the mask, zero outside
    m = texture_mask(32)
    assert not tex[:, :, ~m].any()
    ch = tex[:, :, 0, 0].astype(np.float32)
    assert np.array_equal(tex[:, :, m], np.repeat(ch[:, :, None], int(m.sum()), axis=2).astype(np.float16))
    # the light (last object, emissive 5000) and the walls' uint8 diffuse round trip
    assert np.allclose(ch[-1, 10:13], 5000.0) and np.allclose(ch[:-1, 10:13], 0.0)
    assert np.allclose(ch[0, :3], np.float16(102 / 255)) and np.allclose(ch[:, 7:10], [0.5, 0.5, 1.0])
    # light triangle: tri.obj scaled 2.5 then translated to z = 2.1 (scene_mesh.py:41-55)
    lv, lf = sc.load_obj(os.path.join(os.path.dirname(HERE), "examples", "templates", "lighting", "tri.obj"))
    assert np.allclose(tri[-1], (lv[lf[0]] * 2.5 + [0.0, 0.0, 2.1]).astype(np.float32), atol=1e-6)
    # normals are unit length; planar groups give the plane normal
    assert np.allclose(np.linalg.norm(vn, axis=-1), 1.0, atol=1e-5)
    fn = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    fn /= np.linalg.norm(fn, axis=-1, keepdims=True)
    assert (np.einsum("nkc,nc->nk", vn, fn) > 0.99).all()


def test_look_at_camera_known_answer():
    """to_h5.py:10-34: camera at the position, looking along -z of its frame toward the target, z-up world."""
    c2w = sc.look_at_to_c2w([0.0, -2.0, 0.0], [0.0, 0.0, 0.0], [0.0, 0.0, 1.0])
    assert np.allclose(c2w[:3, 3], [0, -2, 0])
    assert np.allclose(c2w[:3, 2], [0, -1, 0])      # camera backward axis = normalize(position - target)
    assert np.allclose(c2w[:3, 0], [1, 0, 0])       # right = up x backward
    assert np.allclose(c2w[:3, 1], [0, 0, 1])       # up
    assert np.allclose(c2w[:3, :3] @ c2w[:3, :3].T, np.eye(3))


def test_transform_order_rotate_scale_translate():
    t = sc.TransformConfig(translation=[1.0, 0.0, 0.0], rotation=[0.0, 0.0, 90.0], scale=[2.0, 1.0, 1.0],
                           normalize=False)
    v = sc.transform_vertices(np.array([[1.0, 0.0, 0.0]]), t)
    assert np.allclose(v, [[1.0, 1.0, 0.0]])  # rotate (0,1,0), scale x (no effect), translate +x


def test_smooth_shading_cube_and_flat(tmp_path):
    """A cube: 90-degree edges split it into 6 smooth groups whose normals are the face normals."""
    obj = tmp_path / "cube.obj"
    v = [(x, y, z) for x in (0, 1) for y in (0, 1) for z in (0, 1)]
    quads = [(1, 3, 7, 5), (2, 6, 8, 4), (1, 5, 6, 2), (3, 4, 8, 7), (1, 2, 4, 3), (5, 7, 8, 6)]
    obj.write_text("".join(f"v {a} {b} {c}\n" for a, b, c in v) + "".join(f"f {a} {b} {c} {d}\n" for a, b, c, d in quads))
    verts, faces = sc.load_obj(str(obj))
    assert faces.shape == (12, 3)
    groups = sc.smooth_groups(verts, faces)
    assert sorted(len(g) for g in groups) == [2] * 6
    tris, vn, gid = sc.shade(verts, faces, True)
    fn = np.cross(tris[:, 1] - tris[:, 0], tris[:, 2] - tris[:, 0])
    fn /= np.linalg.norm(fn, axis=-1, keepdims=True)
    assert np.allclose(vn, fn[:, None, :].repeat(3, 1))
    t2, vn2, _ = sc.shade(verts, faces, False)
    assert np.allclose(vn2, np.cross(t2[:, 1] - t2[:, 0], t2[:, 2] - t2[:, 0])[:, None, :].repeat(3, 1) /
                       np.linalg.norm(np.cross(t2[:, 1] - t2[:, 0], t2[:, 2] - t2[:, 0]), axis=-1)[:, None, None])


def test_smooth_shading_large_facet_kept_flat():
    """trimesh's smooth_shade facet rule (restated, parity unpinned): a coplanar facet over 1/10 of the mesh
    area next to a gently curved 15-20 degree bend is shaded on its own (plane normals), while without the
    rule the bend (below 30 degrees) joins it into one group and bends its boundary normals."""
    t20, t15 = math.tan(math.radians(20.0)), math.tan(math.radians(15.0))
    v = [(0, 4, 0), (0, 0, 0)]                                              # 0, 1: far corners of the square
    v += [(4, y, 0) for y in range(5)]                                      # 2..6: shared edge x = 4
    v += [(5, y, t20 if y % 2 == 0 else t15) for y in range(5)]             # 7..11: strip's outer edge
    f = [(0, 1, 2)] + [(0, 2 + y, 3 + y) for y in range(4)]                 # flat square (area 16) as a fan
    for y in range(4):
        f += [(2 + y, 7 + y, 8 + y), (2 + y, 8 + y, 3 + y)]                 # strip faces 5..12, not coplanar
    verts, faces = np.asarray(v, dtype=np.float64), np.asarray(f, dtype=np.int64)
    groups = sorted(sorted(g.tolist()) for g in sc.smooth_groups(verts, faces))
    assert groups == [[0, 1, 2, 3, 4], list(range(5, 13))]
    assert len(sc.smooth_groups(verts, faces, facet_minarea=None)) == 1
    tris, vn, _ = sc.shade(verts, faces, True)
    flat = np.isclose(tris[..., 2], 0).all(-1)
    assert flat.sum() == 5 and np.allclose(vn[flat], [0.0, 0.0, 1.0])
    # without the rule the shared-edge vertices average in the strip's normals
    old = sc.FACET_MINAREA
    try:
        sc.FACET_MINAREA = None
        _, vn0, _ = sc.shade(verts, faces, True)
    finally:
        sc.FACET_MINAREA = old
    assert not np.allclose(vn0[flat], [0.0, 0.0, 1.0])


def test_schema_is_strict(tmp_path):
    d = json.load(open(CBOX))
    bad = json.loads(json.dumps(d))
    bad["objects"]["light_0"]["material"]["shininess"] = 1.0
    with pytest.raises(ValueError, match="unexpected"):
        sc._from_dict(sc.SceneConfig, bad)
    bad = json.loads(json.dumps(d))
    del bad["cameras"][0]["fov"]
    with pytest.raises(ValueError, match="missing"):
        sc._from_dict(sc.SceneConfig, bad)
    bad = json.loads(json.dumps(d))
    bad["objects"]["light_0"]["material"]["roughness"] = "rough"
    with pytest.raises(TypeError):
        sc._from_dict(sc.SceneConfig, bad)


@pytest.mark.gpu
def test_cbox_json_to_h5_to_infer_matches_oracle(tmp_path):
    """examples/cbox.json -> cbox.h5 (this converter) -> infer.py on the GPU (v1-base architecture, synthetic
    weights seed 0, 256^2) vs the CPU oracle on the same HDF5 scene: <= 1e-3 relative L2 (north star)."""
    import infer
    from oracle import rf_ref
    from renderformer_amd.config import BASE
    from renderformer_amd.images import read_exr
    from renderformer_amd.weights import synthetic_state_dict
    h5 = sc.convert_scene(CBOX, str(tmp_path / "cbox.h5"))
    out = tmp_path / "out"
    assert infer.main(["--h5_file", h5, "--model_id", "renderformer-v1-base", "--synthetic_seed", "0",
                       "--resolution", "256", "--output_dir", str(out), "--precision", "bf16"]) == 0
    got = read_exr(str(out / "cbox_view_0.exr"))
    d = h5io.load_single_h5_data(h5)
    ref = rf_ref.render(synthetic_state_dict(BASE, seed=0), BASE, d["triangles"][None], d["texture"][None].clone(),
                        d["mask"][None], d["vn"][None], d["c2w"][None], d["fov"][None, :, None], resolution=256)
    ref = ref[0, 0].numpy()
    err = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
    print(f"cbox.json -> h5 -> infer.py vs oracle: rel L2 {err:.3e}")
    assert err < 1e-3


def test_converter_pinned_to_reference_save_to_h5():
    """The package's converter against the reference's own conversion code (tests/golden/make_converter_golden.py
    ran scene_processor.to_h5.save_to_h5 and scene_mesh.normalize_to_unit_sphere from /root/reference with
    data-only stand-ins for trimesh / h5py): per example scene the per-triangle texture channels (material
    packing, channel order, fp16 cast), the x + y <= 32 patch mask, every camera's c2w (look_at_to_c2w) and fov, and
    the unit-sphere normalisation of every normalised object are equal.  Not pinned by this (trimesh absent):
    trimesh's rotation matrices, OBJ round trip and smooth shading — the geometry fed to save_to_h5 is ours."""
    import numpy as np
    from renderformer_amd import scene_convert as sc
    from renderformer_amd.examples import EXAMPLES_DIR, example_names
    from renderformer_amd.scenes import texture_mask
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "converter_examples.npz"))
    names = [n for n in example_names() if f"{n}/c2w" in z.files]
    assert len(names) >= 15
    for name in names:
        cfg = sc.load_scene_config(os.path.join(EXAMPLES_DIR, name + ".json"))
        arr = sc.scene_arrays(cfg, EXAMPLES_DIR)
        ch = arr["texture"][:, :, 0, 0].astype(np.float16)
        assert np.array_equal(ch, z[f"{name}/channels"]), name
        assert int(z[f"{name}/tex_nonzero_outside_mask"]) == 0
        assert np.array_equal(z[f"{name}/mask"], texture_mask(32)), name
        assert np.array_equal(arr["texture"].astype(np.float16)[:, :, ~texture_mask(32)], np.zeros_like(
            arr["texture"][:, :, ~texture_mask(32)], dtype=np.float16))
        np.testing.assert_allclose(arr["c2w"].astype(np.float32), z[f"{name}/c2w"], rtol=0, atol=1e-6, err_msg=name)
        np.testing.assert_array_equal(arr["fov"].astype(np.float32), z[f"{name}/fov"])
        for key, obj in cfg.objects.items():
            k = f"{name}/{key}/normalized"
            if obj.transform.normalize:
                v, _ = sc.load_obj(os.path.join(EXAMPLES_DIR, obj.mesh_path))
                t = sc.TransformConfig(translation=[0.0, 0.0, 0.0], rotation=[0.0, 0.0, 0.0], scale=[1.0, 1.0, 1.0],
                                       normalize=True)
                np.testing.assert_allclose(sc.transform_vertices(v, t), z[k], rtol=0, atol=1e-12, err_msg=k)
