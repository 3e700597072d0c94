"""Stage-1 stream-K attention at the bench shape under the RF_ATTN_DBG ablation builds (timing only).

python tools/attn_ablate.py            -> one line per variant
python tools/attn_ablate.py pmc [reps] -> just the shipped kernel, `reps` launches (for rocprofv3 --pmc)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from renderformer_amd import ops  # noqa: E402
from renderformer_amd._lib import load  # noqa: E402

load()
S, D, H = 5649, 1024, 8
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.randn(S, 3 * D, device="cuda", generator=g).bfloat16()
qs = (qkv[:, :D].float() * ops.Q_LOG2_SCALE).bfloat16()
out = torch.empty(S, D, device="cuda", dtype=torch.bfloat16)
prob = torch.tensor([[0, S, 0, S, 0]], dtype=torch.int32, device="cuda")


def run():
    ops.attention(qs, qkv[:, D:2 * D], qkv[:, 2 * D:], out, prob, S, H, q_prescaled=True)


if len(sys.argv) > 1 and sys.argv[1] == "pmc":
    for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 5):
        run()
    torch.cuda.synchronize()
    sys.exit(0)
fl = 4 * S * S * D
for dbg in ("0", "1", "2", "3", "4", "8", "16", "20", "11", "0"):
    os.environ["RF_ATTN_DBG"] = dbg
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"dbg={dbg:>2}: {ms*1e3:7.1f} us  {fl/ms/1e9:7.1f} TF(equiv)", flush=True)
