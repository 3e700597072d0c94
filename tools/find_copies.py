"""Which host calls launch the small rocclr blit kernels (__amd_rocclr_copyBuffer / fillBuffer) inside a frame?

python tools/find_copies.py   (GPU): renders the bench frame twice, profiles the second with torch.profiler
(with Python stacks) and prints, per blit kernel, the CPU op that launched it and the innermost repo frames."""
import collections
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from renderformer_amd import RenderFormer, RenderFormerRenderingPipeline  # noqa: E402
from renderformer_amd.config import named_config  # noqa: E402
from renderformer_amd.scenes import batch_scenes, synthetic_scene  # noqa: E402
from renderformer_amd.weights import synthetic_state_dict  # noqa: E402

cfg = named_config("large-proxy")
pipe = RenderFormerRenderingPipeline(RenderFormer(cfg, synthetic_state_dict(cfg, seed=0))).to("cuda:0")
b = {k: v.to("cuda:0") for k, v in batch_scenes([synthetic_scene(5633, 1, seed=1)]).items() if k != "tex_channels"}
tex = [b["texture"].clone() for _ in range(3)]


def frame(i):
    return pipe(b["triangles"], tex[i], b["mask"], b["vn"], b["c2w"], b["fov"], resolution=512,
                torch_dtype=torch.bfloat16)


frame(0)
torch.cuda.synchronize()
acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts, with_stack=True) as prof:
    frame(1)
    torch.cuda.synchronize()
evs = prof.events()
by_id = {e.id: e for e in evs}
count = collections.Counter()
for e in evs:
    if e.device_type != torch.autograd.DeviceType.CUDA or "rocclr" not in e.name:
        continue
    parent = e.cpu_parent if getattr(e, "cpu_parent", None) is not None else None
    p = parent
    chain = []
    while p is not None:
        chain.append(p.name)
        p = p.cpu_parent
    stack = []
    for q in ([parent] if parent else []):
        while q is not None and not q.stack:
            q = q.cpu_parent
        if q is not None:
            stack = [s for s in q.stack if "renderformer_amd" in s or "bench" in s or "find_copies" in s][:4]
    count[(e.name[:40], " <- ".join(chain[:4]), " | ".join(stack))] += 1
for (name, chain, stack), n in count.most_common():
    print(f"{n:4d}  {name}  [{chain}]\n        {stack}")
print("kernels in frame:", sum(1 for e in evs if e.device_type == torch.autograd.DeviceType.CUDA))
