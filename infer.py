"""Single-scene CLI, flag-compatible with the reference `infer.py:34-41`.

    python infer.py --h5_file scene.h5 [--model_id DIR|NAME] [--precision bf16|fp16|fp32]
                    [--resolution 512] [--output_dir DIR] [--tone_mapper none]
                    [--synthetic_seed S]

Reads the HDF5 scene with renderformer_amd.h5io (no h5py), renders every view on the HIP
device and writes `{base}_view_{i}.exr` (linear HDR) and `{base}_view_{i}.png` (clip to
[0, 1] x 255) like `infer.py:89-103`.  Offline additions: `--model_id` must be a local
snapshot directory (config.json + model.safetensors) unless `--synthetic_seed` is given, in
which case it names an architecture (e.g. renderformer-v1.1-swin-large) with deterministic
random weights.  Tone mappers other than 'none' need the OCIO configs of `simple_ocio`,
which is not available here, and are rejected.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

from renderformer_amd import RenderFormerRenderingPipeline
from renderformer_amd.h5io import load_single_h5_data
from renderformer_amd.images import hdr_to_ldr, write_exr, write_png

PRECISION = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32}


def add_common_args(parser: argparse.ArgumentParser) -> None:
    parser.add_argument("--model_id", type=str, default="microsoft/renderformer-v1.1-swin-large",
                        help="Local snapshot directory, or an architecture name with --synthetic_seed")
    parser.add_argument("--precision", type=str, choices=["bf16", "fp16", "fp32"], default="fp16")
    parser.add_argument("--resolution", type=int, default=512)
    parser.add_argument("--tone_mapper", type=str, choices=["none", "agx", "filmic", "pbr_neutral"], default="none")
    parser.add_argument("--synthetic_seed", type=int, default=None,
                        help="(offline) random-init weights of the named architecture")


def load_pipeline(args) -> RenderFormerRenderingPipeline:
    if args.tone_mapper != "none":
        raise SystemExit(f"tone mapper {args.tone_mapper!r} needs simple_ocio's OCIO configs (not available); "
                         "use --tone_mapper none")
    model_id = args.model_id
    if args.synthetic_seed is not None and model_id.startswith("microsoft/"):
        model_id = model_id.split("/", 1)[1]
    # "lazy" fp16 range check: the CLIs resolve each frame where they wait for its copy anyway (infer.py: before
    # reading it; batch_infer.py: before the D2H of the next batch), so render never blocks their pipelining
    pipe = RenderFormerRenderingPipeline.from_pretrained(model_id, synthetic_seed=args.synthetic_seed,
                                                         range_check="lazy")
    return pipe.to("cuda")


def save_views(hdr: torch.Tensor, output_dir: str, base_name: str, stages=None) -> list:
    """hdr [nv, H, W, 3] -> {base}_view_{i}.exr / .png (infer.py:89-103).  `stages`: batch_infer.StageTimes."""
    paths = []
    for i in range(hdr.shape[0]):
        img = hdr[i].cpu().numpy().astype("float32")
        hdr_path = os.path.join(output_dir, f"{base_name}_view_{i}.exr")
        ldr_path = os.path.join(output_dir, f"{base_name}_view_{i}.png")
        if stages is None:
            write_exr(hdr_path, img)
            write_png(ldr_path, hdr_to_ldr(img))
        else:
            stages.timed("write: EXR", write_exr, hdr_path, img)
            stages.timed("write: PNG", lambda: write_png(ldr_path, hdr_to_ldr(img)))
        paths += [hdr_path, ldr_path]
    return paths


def main(argv=None):
    parser = argparse.ArgumentParser(description="Infer using triangle radiosity transformer model (MI355X)")
    parser.add_argument("--h5_file", type=str, required=True, help="Path to the input H5 file")
    parser.add_argument("--output_dir", type=str, required=False, help="Output directory (default: next to the H5)")
    add_common_args(parser)
    args = parser.parse_args(argv)

    pipeline = load_pipeline(args)
    data = load_single_h5_data(args.h5_file)
    dev = pipeline.device
    triangles = data["triangles"].unsqueeze(0).to(dev)
    texture = data["texture"].unsqueeze(0).to(dev)
    mask = data["mask"].unsqueeze(0).to(dev)
    vn = data["vn"].unsqueeze(0).to(dev)
    c2w = data["c2w"].unsqueeze(0).to(dev)
    fov = data["fov"].unsqueeze(0).unsqueeze(-1).to(dev)
    imgs = pipeline(triangles=triangles, texture=texture, mask=mask, vn=vn, c2w=c2w, fov=fov,
                    resolution=args.resolution, torch_dtype=PRECISION[args.precision])
    pipeline.resolve(imgs)  # the frame's fp16 range check (re-rendered in place if it overflowed) before reading it
    print("Inference completed. Rendered images shape:", imgs.shape)
    output_dir = args.output_dir if args.output_dir else os.path.dirname(os.path.abspath(args.h5_file))
    os.makedirs(output_dir, exist_ok=True)
    base = os.path.splitext(os.path.basename(args.h5_file))[0]
    for p in save_views(imgs[0], output_dir, base):
        print(f"Saved {p}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
