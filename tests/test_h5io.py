"""HDF5 scene I/O: round trips through our writer, and the reader against files
written by libhdf5 itself where the image has some (PyTables' test data; skipped otherwise)."""
import glob
import os

import numpy as np
import pytest

from renderformer_amd import h5io

LIBHDF5_FILES = "/opt/conda/lib/python3.9/site-packages/tables/tests"


def test_scene_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    n, v = 300, 3
    tri = rng.random((n, 3, 3), dtype=np.float32)
    vn = rng.random((n, 3, 3), dtype=np.float32)
    tex = rng.random((n, 13, 32, 32)).astype(np.float16)
    c2w = rng.random((v, 4, 4), dtype=np.float32)
    fov = np.array([37.5, 40.0, 45.0], np.float32)
    path = str(tmp_path / "scene.h5")
    h5io.write_scene(path, tri, vn, tex, c2w, fov)
    with h5io.File(path) as f:
        assert sorted(f.keys()) == sorted(h5io.SCENE_KEYS)
        assert f["texture"].dtype == np.float16 and f["texture"].shape == tex.shape
        np.testing.assert_array_equal(np.array(f["texture"]), tex)
    d = h5io.load_single_h5_data(path)
    np.testing.assert_array_equal(d["triangles"].numpy(), tri)
    np.testing.assert_array_equal(d["texture"].numpy(), tex.astype(np.float32))
    np.testing.assert_array_equal(d["fov"].numpy(), fov)
    assert d["mask"].dtype.is_floating_point is False and bool(d["mask"].all()) and d["mask"].numel() == n


@pytest.mark.parametrize("dtype", [np.float16, np.float32, np.float64, np.int32, np.int64, np.uint8])
@pytest.mark.parametrize("shape", [(7,), (5, 3), (65, 2, 3), (0, 4)])
def test_dtypes_shapes_chunking(tmp_path, dtype, shape):
    a = (np.arange(int(np.prod(shape))) % 97).astype(dtype).reshape(shape)
    path = str(tmp_path / "x.h5")
    h5io.write_datasets(path, {"a": a, "b": a[::-1].copy()}, max_chunk_bytes=64)  # many chunks, ragged tail
    with h5io.File(path) as f:
        for k, ref in (("a", a), ("b", a[::-1])):
            got = np.array(f[k])
            assert got.dtype == ref.dtype and got.shape == ref.shape
            np.testing.assert_array_equal(got, ref)


def test_uncompressed_and_missing(tmp_path):
    path = str(tmp_path / "u.h5")
    h5io.write_datasets(path, {"fov": np.array([30.0], np.float32)}, compression_level=None)
    with h5io.File(path) as f:
        assert float(np.array(f["fov"])[0]) == 30.0
        with pytest.raises(KeyError):
            f["triangles"]
    bad = tmp_path / "bad.h5"
    bad.write_bytes(b"not hdf5 at all" * 10)
    with pytest.raises(h5io.H5FormatError):
        h5io.File(str(bad))


@pytest.mark.skipif(not os.path.isdir(LIBHDF5_FILES), reason="no libhdf5-written files in this image")
def test_reader_on_libhdf5_files():
    """Files written by libhdf5 (both byte orders, f16/f32/f64, contiguous and chunked): known contents."""
    ref = np.add.outer(np.arange(6), np.arange(5))  # PyTables' smpl_* TestArray: a[i, j] = i + j
    for name in ("i32le", "i32be", "i64le", "i64be", "f64le", "f64be"):
        p = os.path.join(LIBHDF5_FILES, f"smpl_{name}.h5")
        if os.path.exists(p):
            np.testing.assert_array_equal(np.array(h5io.File(p)["TestArray"]), ref)
    p = os.path.join(LIBHDF5_FILES, "float.h5")
    if os.path.exists(p):
        f = h5io.File(p)
        ref = np.add.outer(np.arange(5), np.arange(6)).astype(np.float64)
        for k in ("float16", "float32", "float64"):
            np.testing.assert_array_equal(np.array(f[k]).astype(np.float64), ref)
    # every file either parses or fails with a clear H5FormatError / KeyError (unsupported features)
    for p in glob.glob(os.path.join(LIBHDF5_FILES, "*.h5")):
        try:
            f = h5io.File(p)
        except h5io.H5FormatError:
            continue
        for k in f.keys():
            try:
                np.array(f[k])
            except (h5io.H5FormatError, KeyError):
                pass


@pytest.mark.skipif(h5io._libdeflate() is None, reason="no libdeflate on this machine")
@pytest.mark.parametrize("shape", [(101, 13, 32, 32), (37, 5, 3)])  # 101 rows: a ragged last chunk
def test_libdeflate_matches_zlib(tmp_path, monkeypatch, shape):
    """The libdeflate chunk path (whole chunks inflated into `out`, ragged tail chunks through scratch) reads the
    same bits as zlib, into a fresh array and into read(out=)."""
    rng = np.random.default_rng(1)
    a = (rng.standard_normal(shape) * (rng.random(shape) < 0.3)).astype(np.float16)  # compressible, like textures
    path = str(tmp_path / "t.h5")
    h5io.write_datasets(path, {"t": a}, max_chunk_bytes=1 << 16, compression_level=9)
    got = np.array(h5io.File(path)["t"])
    out = np.full(shape, np.float16(7.0))
    h5io.File(path)["t"].read(out=out)
    monkeypatch.setattr(h5io, "_DEFLATE", False)  # zlib only
    ref = np.array(h5io.File(path)["t"])
    assert np.array_equal(ref.view(np.uint16), a.view(np.uint16))
    assert np.array_equal(got.view(np.uint16), ref.view(np.uint16))
    assert np.array_equal(out.view(np.uint16), ref.view(np.uint16))
