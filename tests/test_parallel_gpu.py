"""The RCCL branch of the frame gather on the GPU (it had never executed anywhere; the gloo
tests take the synchronous host branch).  One process, a one-rank nccl (= RCCL) group on the box's GPU: the
all_gather_into_tensor is issued with async_op=True on RCCL's stream, work is queued behind it on the current
stream (bench.py renders the next frame there), and result() waits through the stream, not the host.  Multi-rank
exchange itself is exercised by the driver's 8-GPU scaling run; the layout logic by the gloo world-2 tests."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import sys, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[2])
from renderformer_amd.parallel import FrameGather
dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{sys.argv[1]}", rank=0, world_size=1)
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
shape = (64, 64, 3)
for ids in ([[0, 1, 2]], [[2, 0, 1]]):  # identity order, and a permutation (index_select after the gather)
    g = FrameGather(ids, shape, dev, collective=True)
    assert g.distributed and not g.gloo
    local = torch.randn(3, *shape, device=dev)
    pend = g.start(local)
    x = torch.randn(2048, 2048, device=dev)
    y = x @ x  # the next step's work, queued on the current stream while the collective is in flight
    out = pend.result()
    exp = torch.empty_like(local)
    exp[torch.tensor(ids[0], device=dev)] = local
    torch.cuda.synchronize()
    assert torch.equal(out, exp), ids
    assert torch.isfinite(y).all()
# the default (no collective for a one-rank group) is the local shortcut
assert not FrameGather([[0, 1]], shape, dev).distributed
dist.destroy_process_group()
print("rccl frame gather ok")
'''


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_frame_gather_rccl_async_one_rank():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", SCRIPT, str(_free_port()), REPO], capture_output=True, text=True,
                       timeout=180, env=env)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0 and "rccl frame gather ok" in r.stdout


SHARDED = r'''
import sys, warnings, torch, torch.distributed as dist
port, repo, rank = sys.argv[1], sys.argv[2], int(sys.argv[3])
sys.path.insert(0, repo)
sys.path.insert(0, repo + "/tests")
from golden_util import load_case, rel_l2
from oracle import rf_ref
from renderformer_amd import RenderFormer, RenderFormerRenderingPipeline
from renderformer_amd.parallel import ShardedRenderer
from test_parity_gpu import _overflow_sd
dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
torch.cuda.set_device(0)
cfg, sd, inp, res, z = load_case("tiny_swin")
big = _overflow_sd(sd)
ref = rf_ref.render(big, cfg, inp["triangles"], inp["texture"].clone(), inp["mask"], inp["vn"], inp["c2w"],
                    inp["fov"], resolution=res)  # [B, V, H, W, 3]
d = {k: v.cuda() for k, v in inp.items()}
B = d["mask"].shape[0]
for mode in ("lazy", "sync"):
    pipe = RenderFormerRenderingPipeline(RenderFormer(cfg, big, range_check=mode)).to("cuda:0")
    sr = ShardedRenderer(pipe, rank, 2)
    scenes = [{k: (v[b:b + 1].clone() if k == "texture" else v[b:b + 1]) for k, v in d.items()} for b in range(B)]
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        frames = sr.render(scenes, res=res)  # scenes over ranks, no resolve by the caller
        views = sr.render_views({k: (v[:1].clone() if k == "texture" else v[:1]) for k, v in d.items()}, res=res)
    for b in range(B):
        err = rel_l2(frames[b].cpu(), ref[b])
        assert torch.isfinite(frames[b]).all() and err < 1e-3, (mode, b, err)
    err = rel_l2(views.cpu(), ref[0])
    assert torch.isfinite(views).all() and err < 1e-3, (mode, "views", err)
    assert pipe.model.range_fallbacks >= 1
dist.barrier()
dist.destroy_process_group()
print(f"rank {rank}: sharded overflow frames ok")
'''


@pytest.mark.timeout(400)
def test_sharded_renderer_resolves_overflowing_frames_gloo_world2():
    """ShardedRenderer.render / render_views under gloo world-2 (two ranks on the box's one GPU)
    with an fp16-overflowing checkpoint and no resolve by the caller: every gathered frame is finite and within 1e-3
    of the oracle, for a lazy model (the renderer resolves each frame before stacking / gathering) and the default
    sync one."""
    port = str(_free_port())
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, "-c", SHARDED, port, REPO, str(r)], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True, env=env) for r in range(2)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=360))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, (p, (o, e)) in enumerate(zip(procs, outs)):
        print(o[-1500:], e[-3000:])
        assert p.returncode == 0 and f"rank {r}: sharded overflow frames ok" in o


def test_batch_copy_streams_run_beside_compute():
    """batch_infer's H2D / D2H side streams come from a probe that keeps only pool streams on a hardware queue other
    than the compute stream's (a shared queue serialized every copy with the frames' kernels: every other
    batch_infer call ran 10-15 % slower); both probe clean, and the pair is reused."""
    import torch
    import batch_infer
    dev = torch.device("cuda")
    compute = torch.cuda.current_stream(dev)
    pair = batch_infer._copy_streams(dev)
    assert len(pair) == 2 and pair is batch_infer._copy_streams(dev)
    for s in pair:
        assert s.cuda_stream != compute.cuda_stream
        assert batch_infer._runs_beside(s, compute)
