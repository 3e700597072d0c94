"""End-to-end batch_infer throughput (BASELINE config 4's data path): HDF5 decode + render + EXR/PNG
writes for a folder of the reference's example scenes (examples/*.json converted by the package's converter,
cycled to n scenes), inline vs pipelined.  python tools/batch_e2e.py [n_scenes] [batch_size]  (GPU box)

Every scene is a new mask pattern for the model, so each pays the per-scene plan (mask read-back + the host
stream-K attention schedule, ~1 ms) that bench.py's repeated frame reuses."""
import json
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import batch_infer  # noqa: E402
from renderformer_amd.examples import convert_all, example_names  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
bs = sys.argv[2] if len(sys.argv) > 2 else "1"
root = tempfile.mkdtemp(prefix="rf_e2e_")
scenes = os.path.join(root, "scenes")
os.makedirs(scenes)
names = example_names()
files = convert_all(names, workers=8, compression_level=9)  # the reference converter's gzip level (to_h5.py:88)
for i in range(n):
    shutil.copy(files[names[i % len(names)]], os.path.join(scenes, f"s{i:03d}_{names[i % len(names)]}.h5"))
args = ["--h5_folder", scenes, "--model_id", "renderformer-v1.1-swin-large", "--synthetic_seed", "0",
        "--resolution", "512", "--batch_size", bs, "--precision", "fp16"]
t = time.perf_counter()
pipe = batch_infer.load_pipeline(batch_infer.argparse.Namespace(tone_mapper="none", model_id="renderformer-v1.1-swin-large",
                                                               synthetic_seed=0))
print(f"model build (synthetic 483.9M-parameter weights + upload): {time.perf_counter() - t:.2f} s", flush=True)
batch_infer.main(args + ["--output_dir", os.path.join(root, "warm")], pipeline=pipe)  # first-touch allocations
res = {}
os.environ["RF_BATCH_PROFILE"] = "1"  # batch_infer.StageTimes: per-stage host time, printed by each run
out_root = tempfile.mkdtemp(prefix="rf_e2e_out_", dir=os.environ.get("RF_E2E_OUTROOT") or root)  # e.g. /dev/shm
for i_pass, mode in enumerate(os.environ.get("RF_E2E_MODES", "0,1,0").split(",")):  # 0 pipelined, 1 inline
    batch_infer.STAGES.t.clear()
    batch_infer.STAGES.n.clear()
    batch_infer.STAGES.on = True
    os.environ["RF_BATCH_INLINE"] = mode
    # RF_E2E_DISTINCT=1: every pass writes new files (a directory of its own) instead of overwriting the last pass's
    out = os.path.join(out_root, "out" + mode + (f"_{i_pass}" if os.environ.get("RF_E2E_DISTINCT") == "1" else ""))
    import torch
    keys = ("num_device_alloc", "num_device_free", "num_alloc_retries", "num_sync_all_streams")
    d0, h0 = torch.cuda.memory_stats(), torch.cuda.host_memory_stats()
    t0 = time.perf_counter()
    batch_infer.main(args + ["--output_dir", out], pipeline=pipe)  # the data path: the model is built once
    dt = time.perf_counter() - t0
    d1, h1 = torch.cuda.memory_stats(), torch.cuda.host_memory_stats()
    print("allocator events in the pass:", json.dumps({**{k: d1.get(k, 0) - d0.get(k, 0) for k in keys},
          **{"host_" + k: h1[k] - h0.get(k, 0) for k in h1 if ("alloc" in k or "free" in k) and "bytes" not in k
             and isinstance(h1[k], (int, float))}}), flush=True)
    key = "inline" if mode == "1" else "pipelined"
    res[key] = max(res.get(key, 0.0), n / dt)
    print(f"{key}: {n / dt:.2f} frames/s end to end ({dt:.2f} s for {n} scenes, batch_size {bs}; model built once "
          f"outside)", flush=True)
print(json.dumps({"batch_infer_e2e_frames_per_s": res, "scenes": n, "batch_size": int(bs), "res": 512,
                  "data": "the reference's 16 example scenes converted to HDF5 (gzip 9), cycled",
                  "host_threads": __import__("renderformer_amd.h5io", fromlist=["host_threads"]).host_threads()}))
shutil.rmtree(out_root, ignore_errors=True)
shutil.rmtree(root, ignore_errors=True)
