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


PRO = ("vn_encoding_proj", "view_transformer.ray_map_encoder")  # bf16 prologue projections (the texture one runs as an fp32 13-wide product)


def make(stage_sel, w_dt, x_dt, a_dt, pro_dt=None):
    def linear(x, sd, name):
        on = stage_sel(name)
        w = sd[name + ".weight"]
        if pro_dt is not None and name in PRO:
            return F.linear(rnd(x, pro_dt), rnd(w, pro_dt), sd.get(name + ".bias"))
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
    import sys as _s
    if "--gpu-like" in _s.argv:  # the GPU path's formats: fp16 GEMMs, bf16 attention, bf16 prologue, fp16 DPT
        _conv, _convt = F.conv2d, F.conv_transpose2d
        for label, dpt16, pro in (("fp16 GEMMs + bf16 attn (as v1 of the emulation)", False, None),
                                  ("  + bf16 prologue GEMMs (vn, texture, ray)", False, bf),
                                  ("  + fp16 DPT conv operands", True, None),
                                  ("  + both (the GPU path's formats)", True, bf)):
            rf_ref.linear, rf_ref._sdpa = make(both, hf, hf, bf, pro)
            if dpt16:
                F.conv2d = lambda x, w, b=None, *a, **k: _conv(rnd(x, hf), rnd(w, hf), b, *a, **k)
                F.conv_transpose2d = lambda x, w, b=None, *a, **k: _convt(rnd(x, hf), rnd(w, hf), b, *a, **k)
            out = run()
            F.conv2d, F.conv_transpose2d = _conv, _convt
            print(f"{label:50s} rel L2 {rel_l2(out, ref):.3e}  AC {rel_l2_ac(out, ref):.3e}", flush=True)
        rf_ref.linear, rf_ref._sdpa = _linear, _sdpa
        return
    if "--dpt" in _s.argv:  # which DPT convolutions' fp16 operands cost the most (GEMMs / prologue fp16, attn bf16)
        _conv, _convt = F.conv2d, F.conv_transpose2d
        pre = "view_transformer.out_dpt."
        groups = {"projects+resize": ("projects", "resize_layers"), "layer_rn": ("_rn",),
                  "refinenets": ("refinenet",), "output_conv1": ("output_conv1",),
                  "output_conv2.0": ("output_conv2.0",)}
        wname = {sd[k].data_ptr(): k for k in sd if k.startswith(pre) and k.endswith(".weight")}
        for label, exempt in [("DPT all fp16 (as the GPU)", ())] + [(f"  ... but {g} exact", v) for g, v in groups.items()]:
            def sel(w):
                n = wname.get(w.data_ptr(), "")
                return n and "output_conv2.2" not in n and not any(e in n for e in exempt)
            F.conv2d = lambda x, w, b=None, *a, **k: _conv(rnd(x, hf if sel(w) else None), rnd(w, hf if sel(w) else None), b, *a, **k)
            F.conv_transpose2d = lambda x, w, b=None, *a, **k: _convt(rnd(x, hf if sel(w) else None), rnd(w, hf if sel(w) else None), b, *a, **k)
            rf_ref.linear, rf_ref._sdpa = make(both, hf, hf, bf, hf)
            out = run()
            F.conv2d, F.conv_transpose2d = _conv, _convt
            print(f"{label:50s} rel L2 {rel_l2(out, ref):.3e}  AC {rel_l2_ac(out, ref):.3e}", flush=True)
        rf_ref.linear, rf_ref._sdpa = _linear, _sdpa
        return
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
