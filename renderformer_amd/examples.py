"""The reference's 16 example scenes (examples/*.json + their OBJ meshes, copied as data) as HDF5 scenes.

BASELINE config 4 is ``batch_infer.py`` over the example scenes (batch_infer.py:102-143); the reference ships
the scene JSONs, not their ``.h5`` files, and converts them with ``scene_processor/convert_scene.py``.  This
module is the regeneration recipe: every scene is converted by the package's own converter
(``scene_convert.convert_scene``: deterministic, no trimesh/h5py) into a cache directory, with gzip level 1
by default (only the file's bytes differ from the reference's level 9, not its data).

    python -m renderformer_amd.examples [out_dir]      # all 16 .h5 files (parallel)
"""
from __future__ import annotations

import hashlib
import os
import re
from concurrent.futures import ProcessPoolExecutor
from typing import Dict, List, Optional

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXAMPLES_DIR = os.path.join(REPO, "examples")


def _natural(s: str):
    return [int(t) if t.isdigit() else t.lower() for t in re.split(r"(\d+)", s)]


def example_names() -> List[str]:
    """The example scenes in natsort order (batch_infer.py:20 sorts the folder with natsort)."""
    return sorted((f[:-5] for f in os.listdir(EXAMPLES_DIR) if f.endswith(".json")), key=_natural)


def cache_dir() -> str:
    return os.environ.get("RF_EXAMPLES_CACHE", os.path.join(os.environ.get("TMPDIR", "/tmp"), "rf_examples_h5"))


def _converter_digest() -> bytes:
    """sha256 of the converter's own sources (scene_convert.py, h5io.py, scenes.py): a converter change (e.g. the
    smooth-shading facet rule) invalidates every cached .h5."""
    h = hashlib.sha256()
    here = os.path.dirname(os.path.abspath(__file__))
    for f in ("scene_convert.py", "h5io.py", "scenes.py"):
        h.update(open(os.path.join(here, f), "rb").read())
    return h.digest()


def _source_digest(name: str) -> str:
    """sha256 of the converter sources, the scene JSON and every OBJ it names: a cached .h5 is reused only when
    all of them are unchanged."""
    import json
    path = os.path.join(EXAMPLES_DIR, name + ".json")
    h = hashlib.sha256(_converter_digest())
    h.update(open(path, "rb").read())
    for obj in json.load(open(path)).get("objects", {}).values():
        h.update(open(os.path.join(EXAMPLES_DIR, obj["mesh_path"]), "rb").read())
    return h.hexdigest()[:16]


def example_h5(name: str, out_dir: Optional[str] = None, compression_level: int = 1) -> str:
    """Path of examples/<name>.json converted to HDF5 (converted on first use, reused while the sources match)."""
    from .scene_convert import convert_scene
    out_dir = out_dir or cache_dir()
    path = os.path.join(out_dir, name + (".h5" if compression_level == 1 else f".gzip{compression_level}.h5"))
    stamp = path + ".src"
    digest = f"{_source_digest(name)}:gzip{compression_level}"
    if not (os.path.exists(path) and os.path.exists(stamp) and open(stamp).read() == digest):
        os.makedirs(out_dir, exist_ok=True)
        tmp = path + f".tmp{os.getpid()}"
        convert_scene(os.path.join(EXAMPLES_DIR, name + ".json"), tmp, compression_level=compression_level)
        os.replace(tmp, path)
        with open(stamp, "w") as f:
            f.write(digest)
    return path


def convert_all(names: Optional[List[str]] = None, out_dir: Optional[str] = None, workers: int = 8,
                compression_level: int = 1) -> Dict[str, str]:
    """Convert several example scenes in parallel processes; returns {name: h5 path}."""
    names = names or example_names()
    out_dir = out_dir or cache_dir()
    workers = max(1, min(workers, len(names)))
    if workers == 1:
        return {n: example_h5(n, out_dir, compression_level) for n in names}
    with ProcessPoolExecutor(workers) as ex:
        futs = {n: ex.submit(example_h5, n, out_dir, compression_level) for n in names}
        return {n: f.result() for n, f in futs.items()}


def scene_inputs(name: str) -> Dict[str, np.ndarray]:
    """The scene's tensors exactly as an HDF5 reader returns them (float32; the texture's per-triangle channel
    constants rounded through fp16 like to_h5's f16 texture), without the 32x32 patches: triangles [N,3,3],
    vn [N,3,3], tex_channels [N,13], c2w [V,4,4], fov [V]."""
    from .scene_convert import load_scene_config, object_arrays
    cfg = load_scene_config(os.path.join(EXAMPLES_DIR, name + ".json"))
    tris, vns, chs = [], [], []
    for obj in cfg.objects.values():
        t, n, c = object_arrays(obj, EXAMPLES_DIR)
        tris.append(t)
        vns.append(n)
        chs.append(c)
    from .scenes import look_at_to_c2w
    return {
        "triangles": np.concatenate(tris).astype(np.float32),
        "vn": np.concatenate(vns).astype(np.float32),
        "tex_channels": np.concatenate(chs).astype(np.float16).astype(np.float32),
        "c2w": np.stack([look_at_to_c2w(c.position, c.look_at, c.up) for c in cfg.cameras]).astype(np.float32),
        "fov": np.array([c.fov for c in cfg.cameras], dtype=np.float32),
    }


def inputs_digest(arrays: Dict[str, np.ndarray]) -> str:
    """sha256 over the scene tensors' bytes (fixtures record it: the converter's output is pinned with them)."""
    h = hashlib.sha256()
    for k in ("triangles", "vn", "tex_channels", "c2w", "fov"):
        a = np.ascontiguousarray(arrays[k])
        h.update(k.encode())
        h.update(str(a.dtype).encode())
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()[:32]


if __name__ == "__main__":
    import sys
    import time
    t0 = time.time()
    out = convert_all(out_dir=sys.argv[1] if len(sys.argv) > 1 else None)
    for n, p in out.items():
        print(f"{n}: {p}")
    print(f"{len(out)} scenes in {time.time() - t0:.1f} s")
