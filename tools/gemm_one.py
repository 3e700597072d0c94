"""Run one GEMM shape repeatedly (for rocprofv3 --pmc):  python tools/gemm_one.py M N K [epi] [reps]"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from renderformer_amd import ops  # noqa: E402

m, n, k = (int(x) for x in sys.argv[1:4])
epi = int(sys.argv[4]) if len(sys.argv) > 4 else ops.EPI_BF16
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 20
a = torch.randn(m, k, device="cuda").bfloat16()
w = (torch.randn(n, k, device="cuda") / math.sqrt(k)).bfloat16()
c = torch.empty(m, n if epi != ops.EPI_SWIGLU else n // 2, device="cuda",
                dtype=torch.bfloat16 if epi in (ops.EPI_BF16, ops.EPI_SWIGLU) else torch.float32)
for _ in range(reps):
    ops.gemm(a, w, c, None, epi)
torch.cuda.synchronize()
