"""Per-projection error of the MX fp8 stage-2 mode against the reference fixtures.

    python tools/fp8_study.py [case ...]        (GPU; default: large_cbox_r512 large_cbox_r1024_v4)

For each subset of the stage-2 projections put in MX fp8 (RF_FP8_PROJ), renders the fixture scene through the
drop-in pipeline and prints the HDR rel L2 (and on the deviation from the mean) against the reference render.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]

import torch  # noqa: E402

from golden_util import load_case, reference_hdr, rel_l2, rel_l2_ac  # noqa: E402

SUBSETS = ["f16", None, "q", "out", "self_in", "self_out", "w13", "w2", "w13,w2", "q,out,self_in,self_out",
           "q,out,self_in,self_out,w13,w2"]


def main():
    from renderformer_amd import RenderFormer, RenderFormerRenderingPipeline
    cases = sys.argv[1:] or ["large_cbox_r512", "large_cbox_r1024_v4"]
    res_all = {}
    for name in cases:
        cfg, sd, inp, res, z = load_case(name)
        ref, st = reference_hdr(z)
        d = {k: v.cuda() for k, v in inp.items()}
        for sub in SUBSETS:
            # "f16": the default fp16 projection operands; None: bf16 operands (the base the fp8 mode runs on)
            fp8 = sub not in ("f16", None)
            if fp8:
                os.environ["RF_FP8_PROJ"] = sub
            else:
                os.environ.pop("RF_FP8_PROJ", None)
            operands = "f16" if sub == "f16" else "bf16"
            pipe = RenderFormerRenderingPipeline(RenderFormer(cfg, sd, fp8=fp8, operands=operands)).to("cuda")
            out = pipe(d["triangles"], d["texture"].clone(), d["mask"], d["vn"], d["c2w"], d["fov"], resolution=res)
            got = out[:, :, ::st, ::st].cpu()
            e, ac = rel_l2(got, ref), rel_l2_ac(got, ref)
            res_all[f"{name}/{sub or 'bf16'}"] = (e, ac)
            print(f"{name} fp8[{sub or 'none (bf16)'}]: rel L2 {e:.3e}  deviation-from-mean {ac:.3e}", flush=True)
            del pipe, out
            torch.cuda.empty_cache()
    print(json.dumps(res_all))


if __name__ == "__main__":
    main()
