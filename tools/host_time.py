"""Host enqueue time of one bench frame vs its GPU time: is the frame host-bound?
python tools/host_time.py [new]   (GPU box)
new: every frame a NEW mask pattern (batch_infer's case: one plan per scene), and a cProfile of those renders' host
time (the 25 functions with the most cumulative time)."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from renderformer_amd import RenderFormer, RenderFormerRenderingPipeline  # noqa: E402
from renderformer_amd.config import named_config  # noqa: E402
from renderformer_amd.scenes import batch_scenes, synthetic_scene  # noqa: E402
from renderformer_amd.weights import synthetic_state_dict  # noqa: E402

new = len(sys.argv) > 1 and sys.argv[1] == "new"
cfg = named_config("large-proxy")
# lazy range check: render returns after enqueueing (the default "sync" waits for the frame's end event)
pipe = RenderFormerRenderingPipeline(RenderFormer(cfg, synthetic_state_dict(cfg, seed=0), range_check="lazy")).to("cuda")
scenes = [{k: v.cuda() for k, v in batch_scenes([synthetic_scene(n, 1, seed=1)]).items() if k != "tex_channels"}
          for n in ((5633, 5401, 5702, 5555, 5633, 5480, 5610, 5599, 5500, 5650, 5633, 5377) if new else (5633,))]
hosts = [s["mask"].cpu().numpy() for s in scenes]
texs = [scenes[i % len(scenes)]["texture"].clone() for i in range(12)]


def frame(i):
    b = scenes[i % len(scenes)]
    if new:
        pipe.model.plan_hint(b["mask"], hosts[i % len(scenes)])  # batch_infer's path: no mask read-back
    return pipe(b["triangles"], texs[i], b["mask"], b["vn"], b["c2w"], b["fov"], resolution=512,
                torch_dtype=torch.bfloat16)


for i in range(3):
    frame(i)
torch.cuda.synchronize()
for i in range(3, 8):
    t0 = time.perf_counter()
    frame(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"frame: host enqueue {1e3*(t1-t0):.2f} ms, enqueue+drain {1e3*(t2-t0):.2f} ms", flush=True)
t0 = time.perf_counter()
prof = cProfile.Profile() if new else None
if prof:
    prof.enable()
for i in range(8, 12):
    frame(i)
if prof:
    prof.disable()
torch.cuda.synchronize()
print(f"4 back-to-back frames: {1e3*(time.perf_counter()-t0)/4:.2f} ms/frame")
if prof:
    pstats.Stats(prof).sort_stats("cumulative").print_stats(25)
pipe.resolve()
