"""End-to-end batch_infer throughput: HDF5 decode + render + EXR/PNG writes for a
folder of cbox-sized synthetic scenes, inline vs pipelined.  python tools/batch_e2e.py [n_scenes]  (GPU box)"""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import batch_infer  # noqa: E402
from renderformer_amd import h5io  # noqa: E402
from renderformer_amd.scenes import expand_texture, synthetic_scene  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
root = tempfile.mkdtemp(prefix="rf_e2e_")
scenes = os.path.join(root, "scenes")
os.makedirs(scenes)
for i in range(n):
    sc = synthetic_scene(5633, 1, seed=100 + i)
    h5io.write_scene(os.path.join(scenes, f"s{i}.h5"), sc.triangles, sc.vn,
                     expand_texture(sc.tex_channels).astype(np.float16), sc.c2w, sc.fov)
args = ["--h5_folder", scenes, "--model_id", "renderformer-v1.1-swin-large", "--synthetic_seed", "0",
        "--resolution", "512", "--batch_size", "1", "--precision", "bf16"]
batch_infer.main(args + ["--output_dir", os.path.join(root, "warm")])  # build + tune
for mode in ("1", "0", "1", "0"):
    os.environ["RF_BATCH_INLINE"] = mode
    t0 = time.perf_counter()
    batch_infer.main(args + ["--output_dir", os.path.join(root, "out" + mode)])
    dt = time.perf_counter() - t0
    print(f"{'inline' if mode == '1' else 'pipelined'}: {n / dt:.2f} frames/s end to end ({dt:.2f} s for {n})",
          flush=True)
