"""Host enqueue time of one bench frame vs its GPU time: is the frame host-bound?
python tools/host_time.py   (GPU box)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from renderformer_amd import RenderFormer, RenderFormerRenderingPipeline  # noqa: E402
from renderformer_amd.config import named_config  # noqa: E402
from renderformer_amd.scenes import batch_scenes, synthetic_scene  # noqa: E402
from renderformer_amd.weights import synthetic_state_dict  # noqa: E402

cfg = named_config("large-proxy")
pipe = RenderFormerRenderingPipeline(RenderFormer(cfg, synthetic_state_dict(cfg, seed=0))).to("cuda")
b = {k: v.cuda() for k, v in batch_scenes([synthetic_scene(5633, 1, seed=1)]).items() if k != "tex_channels"}
texs = [b["texture"].clone() for _ in range(12)]


def frame(i):
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
for i in range(8, 12):
    frame(i)
torch.cuda.synchronize()
print(f"4 back-to-back frames: {1e3*(time.perf_counter()-t0)/4:.2f} ms/frame")
