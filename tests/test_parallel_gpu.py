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
