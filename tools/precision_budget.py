"""Where the bf16 path's HDR error comes from: the CPU oracle with operands rounded to bf16 / fp16 at chosen
places (GEMM weights, GEMM inputs, attention q/k/v and P), per stage, vs the plain fp32 oracle.

    python tools/precision_budget.py [case]     (CPU; default large_cbox_r512)

Each line: variant, rel L2 and rel L2 of the deviation from the mean (the tests' rel_l2_ac) vs fp32.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from golden_util import load_case, rel_l2, rel_l2_ac  # noqa: E402
from oracle import rf_ref  # noqa: E402

_linear, _sdpa = rf_ref.linear, rf_ref._sdpa
STATE = {"stage": None}


def rnd(t, dt):
    return t if dt is None else t.to(dt).float()


def make(stage_sel, w_dt, x_dt, a_dt):
    def linear(x, sd, name):
        on = stage_sel(name)
        w = sd[name + ".weight"]
        return F.linear(rnd(x, x_dt if on else None), rnd(w, w_dt if on else None), sd.get(name + ".bias"))

    def sdpa(q, k, v, mask):
        on = stage_sel(STATE["stage"] or "")
        if not on or a_dt is None:
            return _sdpa(q, k, v, mask)
        q, k, v = rnd(q, a_dt), rnd(k, a_dt), rnd(v, a_dt)
        s = q @ k.transpose(-1, -2) / q.shape[-1] ** 0.5
        if mask is not None:
            s = s.masked_fill(~mask, float("-inf")) if mask.dtype == torch.bool else s + mask
        m = s.amax(-1, keepdim=True)
        p = torch.exp(s - m)
        l = p.sum(-1, keepdim=True)
        return (rnd(p, a_dt) @ v) / l
    return linear, sdpa


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "large_cbox_r512"
    cfg, sd, inp, res, z = load_case(name)
    torch.set_num_threads(os.cpu_count() or 8)

    def run():
        return rf_ref.render(sd, cfg, inp["triangles"], inp["texture"].clone(), inp["mask"], inp["vn"], inp["c2w"],
                             inp["fov"], res)

    # tag attention calls with the stage they belong to (mha's projection names carry it)
    orig_mha = rf_ref.mha

    def mha(sd_, p, *a, **k):
        STATE["stage"] = p
        return orig_mha(sd_, p, *a, **k)
    rf_ref.mha = mha
    ref = run()
    s1 = lambda n: n.startswith("transformer.")  # noqa: E731
    s2 = lambda n: n.startswith("view_transformer.transformer.")  # noqa: E731
    both = lambda n: s1(n) or s2(n)  # noqa: E731
    bf, hf = torch.bfloat16, torch.float16
    variants = [
        ("bf16 all (stage 1 + 2: W, X, attn)", both, bf, bf, bf),
        ("bf16 stage 1 only", s1, bf, bf, bf),
        ("bf16 stage 2 only", s2, bf, bf, bf),
        ("bf16 stage 2 weights only", s2, bf, None, None),
        ("bf16 stage 2 GEMM inputs only", s2, None, bf, None),
        ("bf16 stage 2 attention only", s2, None, None, bf),
        ("fp16 all", both, hf, hf, hf),
        ("fp16 W+X, bf16 attn", both, hf, hf, bf),
        ("bf16 W, fp16 X+attn", both, bf, hf, hf),
    ]
    for label, sel, w, x, a in variants:
        rf_ref.linear, rf_ref._sdpa = make(sel, w, x, a)
        out = run()
        print(f"{label:45s} rel L2 {rel_l2(out, ref):.3e}  AC {rel_l2_ac(out, ref):.3e}", flush=True)
    rf_ref.linear, rf_ref._sdpa = _linear, _sdpa


if __name__ == "__main__":
    main()
