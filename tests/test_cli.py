"""infer.py / batch_infer.py (reference CLIs) and the image writers."""
import json
import os
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from golden_util import load_case, rel_l2  # noqa: E402
from renderformer_amd import h5io  # noqa: E402
from renderformer_amd.images import hdr_to_ldr, read_exr, read_png, write_exr, write_png  # noqa: E402


def test_exr_png_roundtrip(tmp_path):
    rng = np.random.default_rng(1)
    hdr = (rng.standard_normal((17, 23, 3)) * 100).astype(np.float32)
    write_exr(str(tmp_path / "a.exr"), hdr)
    np.testing.assert_array_equal(read_exr(str(tmp_path / "a.exr")), hdr)
    ldr = hdr_to_ldr(hdr)
    assert ldr.dtype == np.uint8 and ldr.max() <= 255
    write_png(str(tmp_path / "a.png"), ldr)
    np.testing.assert_array_equal(read_png(str(tmp_path / "a.png")), ldr)
    with open(tmp_path / "a.exr", "rb") as f:
        assert f.read(4) == bytes([0x76, 0x2F, 0x31, 0x01])  # OpenEXR magic
    with open(tmp_path / "a.png", "rb") as f:
        assert f.read(8) == b"\x89PNG\r\n\x1a\n"


def test_natural_sort_padding_and_collate(tmp_path):
    import batch_infer
    names = ["s10.h5", "s2.h5", "s1.h5", "S3.h5"]
    assert sorted(names, key=batch_infer.natural_key) == ["s1.h5", "s2.h5", "S3.h5", "s10.h5"]
    rng = np.random.default_rng(0)
    for i, n in enumerate((5, 9)):
        h5io.write_scene(str(tmp_path / f"s{i}.h5"), rng.random((n, 3, 3)), rng.random((n, 3, 3)),
                         rng.random((n, 13, 32, 32)), rng.random((2, 4, 4)), [37.5, 40.0])
    a = batch_infer.load_scene(str(tmp_path / "s0.h5"), padding_length=12)
    assert a["triangles"].shape == (12, 3, 3) and int(a["mask"].sum()) == 5 and not a["mask"][5:].any()
    assert float(a["texture"][5:].abs().sum()) == 0.0
    b = batch_infer.load_scene(str(tmp_path / "s1.h5"), padding_length=12)
    assert batch_infer.collate([a, b])["texture"].shape == (2, 12, 13, 32, 32)
    with pytest.raises(ValueError):
        batch_infer.collate([batch_infer.load_scene(str(tmp_path / "s0.h5")),
                             batch_infer.load_scene(str(tmp_path / "s1.h5"))])
    with pytest.raises(ValueError):
        batch_infer.load_scene(str(tmp_path / "s1.h5"), padding_length=4)


def test_cli_rejects_unavailable_tone_mapper(tmp_path):
    import infer
    with pytest.raises(SystemExit):
        infer.main(["--h5_file", str(tmp_path / "x.h5"), "--tone_mapper", "agx", "--model_id", "x"])


def _snapshot_and_scene(tmp_path, tex_dtype=np.float16):
    """tiny_swin golden: local snapshot dir (config.json + model.safetensors) + its scene 0 (valid triangles
    only; the reference output is padding-invariant) as an HDF5 file."""
    from safetensors.torch import save_file
    cfg, sd, inp, res, z = load_case("tiny_swin")
    snap = tmp_path / "snap"
    snap.mkdir()
    (snap / "config.json").write_text(json.dumps(cfg.to_dict()))
    save_file({k: v.contiguous() for k, v in sd.items()}, str(snap / "model.safetensors"))
    m = inp["mask"][0].numpy().astype(bool)
    h5 = tmp_path / "scenes" / "tiny.h5"
    h5.parent.mkdir()
    h5io.write_scene(str(h5), inp["triangles"][0].numpy()[m], inp["vn"][0].numpy()[m],
                     inp["texture"][0].numpy()[m].astype(tex_dtype), inp["c2w"][0].numpy(),
                     inp["fov"][0].numpy().reshape(-1), texture_dtype=tex_dtype)
    return snap, h5, res, z


@pytest.mark.gpu
def test_infer_cli_matches_reference(tmp_path):
    import infer
    snap, h5, res, z = _snapshot_and_scene(tmp_path)
    out = tmp_path / "out"
    assert infer.main(["--h5_file", str(h5), "--model_id", str(snap), "--resolution", str(res),
                       "--output_dir", str(out)]) == 0
    nv = z["hdr"].shape[1]
    for i in range(nv):
        hdr = read_exr(str(out / f"tiny_view_{i}.exr"))
        assert rel_l2(hdr, z["hdr"][0, i]) < 1e-3
        np.testing.assert_array_equal(read_png(str(out / f"tiny_view_{i}.png")), hdr_to_ldr(hdr))


@pytest.mark.gpu
def test_batch_infer_cli(tmp_path):
    import batch_infer
    snap, h5, res, z = _snapshot_and_scene(tmp_path)
    os.link(h5, h5.parent / "tiny2.h5")
    out = tmp_path / "out"
    assert batch_infer.main(["--h5_folder", str(h5.parent), "--model_id", str(snap), "--resolution", str(res),
                             "--output_dir", str(out), "--batch_size", "2"]) == 0
    a = read_exr(str(out / "tiny_view_0.exr"))
    b = read_exr(str(out / "tiny2_view_0.exr"))
    # same scene twice in one batch: fp32 sum order may differ per image (stream-K K ranges, KV split), and
    # the fp16 DPT operand planes turn such last-bit differences into occasional fp16 ulp flips (~2e-5)
    assert rel_l2(a, b) < 1e-4
    assert rel_l2(a, z["hdr"][0, 0]) < 1e-3


def test_load_scene_keeps_file_texture_dtype(tmp_path):
    """The pipelined loader keeps the texture dtype the file stores (fp16 from to_h5, fp32 from other writers):
    an fp32 texture must not be rounded through fp16 on the way to the device."""
    import batch_infer
    rng = np.random.default_rng(3)
    for dt in (np.float16, np.float32):
        p = str(tmp_path / f"s_{np.dtype(dt).name}.h5")
        tex = (rng.random((4, 13, 32, 32)) * 3).astype(dt)
        h5io.write_scene(p, rng.random((4, 3, 3)), rng.random((4, 3, 3)), tex, rng.random((1, 4, 4)), [40.0],
                         texture_dtype=dt)
        kept = batch_infer.load_scene(p, texture_dtype=None)["texture"]
        assert kept.dtype == torch.from_numpy(tex).dtype
        np.testing.assert_array_equal(kept.numpy(), tex)
        np.testing.assert_array_equal(batch_infer.load_scene(p)["texture"].numpy(), tex.astype(np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("tex_dtype", [np.float16, np.float32])
def test_batch_infer_pipelined_matches_inline(tmp_path, monkeypatch, tex_dtype):
    """The pipelined data path (loader thread, pinned H2D/D2H side streams) writes the same images as the
    inline loop, over several batches (3 scenes, batch size 1: every overlap case), for fp16 and fp32 files."""
    import batch_infer
    snap, h5, res, z = _snapshot_and_scene(tmp_path, tex_dtype)
    for i in (2, 3):
        os.link(h5, h5.parent / f"tiny{i}.h5")
    outs = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("RF_BATCH_INLINE", mode)
        out = tmp_path / f"out{mode}"
        assert batch_infer.main(["--h5_folder", str(h5.parent), "--model_id", str(snap), "--resolution", str(res),
                                 "--output_dir", str(out), "--batch_size", "1"]) == 0
        outs[mode] = out
    for name in ("tiny", "tiny2", "tiny3"):
        a = read_exr(str(outs["1"] / f"{name}_view_0.exr"))
        b = read_exr(str(outs["0"] / f"{name}_view_0.exr"))
        assert rel_l2(a, b) < 1e-4  # (fp32 sum-order differences only, as in test_batch_infer_cli)
        assert rel_l2(a, z["hdr"][0, 0]) < 1e-3


def test_batch_loader_decodes_into_pinned_slots_like_collate(tmp_path):
    """batch_infer's pipelined loader decodes each scene straight into its slot of the batch tensors (h5io
    read(out=), no collate / pin copies): same tensors as collate(load_scene(...)) for equal-N batches and with
    --padding_length (zero padding rows, mask False), in the file's texture dtype."""
    import numpy as np
    import batch_infer
    from renderformer_amd.h5io import write_scene
    rng = np.random.default_rng(3)
    paths = []
    for i, n in enumerate((37, 37, 20)):
        p = str(tmp_path / f"s{i}.h5")
        tex = rng.random((n, 13, 32, 32), dtype=np.float32)
        write_scene(p, rng.random((n, 3, 3)), rng.random((n, 3, 3)), tex, rng.random((2, 4, 4)),
                    rng.random(2) * 40 + 20)
        paths.append(p)
    for idx, pad in (([0, 1], None), ([0, 2], 64), ([2], None)):
        _, got = batch_infer._load_batch_pinned(paths, idx, pad, pinned=False)
        ref = batch_infer.collate([batch_infer.load_scene(paths[i], pad, None) for i in idx])
        assert set(got) == set(ref)
        for k in ref:
            assert got[k].dtype == ref[k].dtype and got[k].shape == ref[k].shape, k
            assert torch.equal(got[k], ref[k]), k
    with pytest.raises(ValueError, match="padding_length"):
        batch_infer._load_batch_pinned(paths, [0, 2], None, pinned=False)
