"""Folder CLI, flag-compatible with the reference `batch_infer.py:62-75`.

    python batch_infer.py --h5_folder DIR [--batch_size 8] [--padding_length N] [--num_workers 0]
                          [--output_dir DIR] [--save_video] + the infer.py model flags

Scenes are read with renderformer_amd.h5io in natural-sort order (`batch_infer.py:19-21`),
padded to `--padding_length` with an explicit mask when given (`:36-45`), batched by
`--batch_size` and rendered; outputs are `{base}_view_{i}.exr/.png` as in `:145-163`.
Under `torch.distributed.run` (one process per GPU) every rank renders its longest-
processing-time share of the scenes (renderformer_amd.parallel.assign_units on the FLOP
model); no data crosses ranks.  `--save_video` needs an mp4 encoder (imageio/ffmpeg) that
the image lacks: frames are written as PNGs and the video step is skipped with a notice.
"""
from __future__ import annotations

import argparse
import glob
import os
import re
import sys

import numpy as np
import torch

from infer import PRECISION, add_common_args, load_pipeline, save_views
from renderformer_amd.h5io import File
from renderformer_amd.parallel import assign_units, scene_cost


def natural_key(path: str):
    """natsort's default ordering for the file names used here (digit runs compare numerically)."""
    return [int(t) if t.isdigit() else t.lower() for t in re.split(r"(\d+)", path)]


def load_scene(path: str, padding_length=None) -> dict:
    """`TriangleRenderH5Dataset.__getitem__` (batch_infer.py:27-58)."""
    with File(path) as f:
        tri = torch.from_numpy(np.array(f["triangles"])).float()
        tex = torch.from_numpy(np.array(f["texture"])).float()
        vn = torch.from_numpy(np.array(f["vn"])).float()
        c2w = torch.from_numpy(np.array(f["c2w"]).astype(np.float32))
        fov = torch.from_numpy(np.array(f["fov"]).astype(np.float32))
    n = tri.shape[0]
    if padding_length is not None:
        if padding_length < n:
            raise ValueError(f"{path}: {n} triangles exceed --padding_length {padding_length}")
        pad = padding_length - n
        tri = torch.cat((tri, tri.new_zeros((pad,) + tri.shape[1:])))
        tex = torch.cat((tex, tex.new_zeros((pad,) + tex.shape[1:])))
        vn = torch.cat((vn, vn.new_zeros((pad,) + vn.shape[1:])))
        mask = torch.zeros(padding_length, dtype=torch.bool)
        mask[:n] = True
    else:
        mask = torch.ones(n, dtype=torch.bool)
    return {"triangles": tri, "texture": tex, "mask": mask, "c2w": c2w, "fov": fov, "vn": vn, "file_path": path}


def collate(items):
    keys = ("triangles", "texture", "mask", "c2w", "fov", "vn")
    shapes = {k: {tuple(it[k].shape) for it in items} for k in keys}
    if any(len(s) > 1 for s in shapes.values()):
        raise ValueError("scenes in one batch differ in shape: pass --padding_length (as the reference requires)")
    return {k: torch.stack([it[k] for it in items]) for k in keys}


def main(argv=None):
    parser = argparse.ArgumentParser(description="Batch inference using triangle radiosity transformer model (MI355X)")
    parser.add_argument("--h5_folder", type=str, required=True)
    parser.add_argument("--batch_size", type=int, default=8)
    parser.add_argument("--padding_length", type=int, default=None)
    parser.add_argument("--num_workers", type=int, default=0, help="accepted for compatibility; loading is inline")
    parser.add_argument("--output_dir", type=str, default=None)
    parser.add_argument("--save_video", action="store_true", default=True)
    add_common_args(parser)
    args = parser.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    files = sorted(glob.glob(os.path.join(args.h5_folder, "*.h5")), key=natural_key)
    print(f"Found {len(files)} h5 files in {args.h5_folder}")
    pipeline = load_pipeline(args)
    cfg = pipeline.config
    if world > 1:
        costs = []
        for p in files:
            with File(p) as f:
                costs.append(scene_cost(cfg, f["triangles"].shape[0], f["c2w"].shape[0], args.resolution))
        mine = assign_units(costs, world)[rank]
    else:
        mine = list(range(len(files)))
    output_dir = args.output_dir if args.output_dir is not None else args.h5_folder
    os.makedirs(output_dir, exist_ok=True)
    dev = pipeline.device
    n_frames = 0
    for b0 in range(0, len(mine), args.batch_size):
        items = [load_scene(files[i], args.padding_length) for i in mine[b0:b0 + args.batch_size]]
        batch = {k: v.to(dev) for k, v in collate(items).items()}
        imgs = pipeline(triangles=batch["triangles"], texture=batch["texture"], mask=batch["mask"], vn=batch["vn"],
                        c2w=batch["c2w"], fov=batch["fov"].unsqueeze(-1), resolution=args.resolution,
                        torch_dtype=PRECISION[args.precision])
        for i, it in enumerate(items):
            base = os.path.splitext(os.path.basename(it["file_path"]))[0]
            save_views(imgs[i], output_dir, base)
            n_frames += imgs.shape[1]
    print(f"Output saved to: {output_dir} ({n_frames} frames on rank {rank}/{world})")
    if args.save_video:
        print("video.mp4 not written: no mp4 encoder in this environment (frames are saved as PNG)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
