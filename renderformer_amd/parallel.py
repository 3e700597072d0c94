"""Multi-GPU rendering: one process per GPU, (scene, view) frames sharded across ranks.

The north-star path shards naturally: frames are independent
(a view rendered alone equals the same view inside a batch), so ranks render
disjoint units with no collective on the data path.  Scenes differ a lot in
cost (N from ~0.5k to ~12k triangles, stage 1 is O(S^2)), so units are assigned
by greedy longest-processing-time on the analytic FLOP model, not round-robin.
The only collective is the optional gather of finished HDR frames to every
rank (RCCL all_gather over xGMI on GPUs, gloo in the CPU tests).
"""
from __future__ import annotations

import heapq
from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist

from .config import RenderFormerConfig
from .flops import frame_flops


def scene_cost(cfg: RenderFormerConfig, n_tris: int, n_views: int, res: int) -> float:
    """Algorithmic FLOPs to render all views of one scene (stage 1 once, stage 2 + DPT per view)."""
    return float(frame_flops(cfg, n_tris, res, n_views)["total"])


def assign_units(costs: Sequence[float], world: int) -> List[List[int]]:
    """Greedy LPT: heaviest unit first onto the least-loaded rank (ties -> lowest rank). Deterministic."""
    if world < 1:
        raise ValueError("world must be >= 1")
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    heap: List[Tuple[float, int]] = [(0.0, r) for r in range(world)]
    out: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + costs[i], r))
    for lst in out:
        lst.sort()
    return out


def max_over_ranks(value: float, device=None) -> float:
    """bench.py timing rule: the job time is the slowest rank's."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_frames(local: torch.Tensor, local_ids: Sequence[int], n_total: int) -> torch.Tensor:
    """all_gather per-rank frame stacks [n_local, ...] into [n_total, ...] in global unit order.

    Every rank must call it, including ranks with no units (n_local = 0, but the trailing frame shape
    still given): the collective needs every member.  On RCCL the frames stay on the device (xGMI);
    under gloo (CPU tests) device tensors are moved to the host for the exchange."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        out = local.new_empty((n_total,) + tuple(local.shape[1:]))
        if len(local_ids):
            out[torch.as_tensor(list(local_ids), dtype=torch.long, device=local.device)] = local
        return out
    world = dist.get_world_size()
    dev = local.device
    xdev = torch.device("cpu") if dist.get_backend() == "gloo" else dev
    n_loc = torch.tensor([local.shape[0]], device=xdev)
    counts = [torch.zeros_like(n_loc) for _ in range(world)]
    dist.all_gather(counts, n_loc)
    cmax = int(max(int(c.item()) for c in counts))
    if cmax == 0:
        return local.new_empty((n_total,) + tuple(local.shape[1:]))
    pad = torch.zeros((cmax,) + tuple(local.shape[1:]), dtype=local.dtype, device=xdev)
    pad[: local.shape[0]] = local.to(xdev)
    ids = torch.full((cmax,), -1, dtype=torch.long, device=xdev)
    if len(local_ids):
        ids[: len(local_ids)] = torch.as_tensor(list(local_ids), dtype=torch.long, device=xdev)
    bufs = [torch.empty_like(pad) for _ in range(world)]
    id_bufs = [torch.empty_like(ids) for _ in range(world)]
    dist.all_gather(bufs, pad)
    dist.all_gather(id_bufs, ids)
    out = torch.empty((n_total,) + tuple(local.shape[1:]), dtype=local.dtype, device=xdev)
    for b, i in zip(bufs, id_bufs):
        keep = i >= 0
        out[i[keep]] = b[keep]
    return out.to(dev)


def shard_views(n_views: int, world: int) -> List[range]:
    """Contiguous view ranges of ONE scene per rank (single scene with many views): views are
    independent given the scene (a view rendered alone == the same view in a batch), so rank r renders
    views [start_r, end_r) with stage 1 recomputed locally (2-5 TFLOP, ~2 ms) instead of broadcast."""
    if world < 1:
        raise ValueError("world must be >= 1")
    return [range(n_views * r // world, n_views * (r + 1) // world) for r in range(world)]


def frame_channels(cfg: RenderFormerConfig) -> int:
    return 4 if cfg.include_alpha else 3


class ShardedRenderer:
    """Render a list of scenes across ranks: each rank runs the pipeline on its LPT share, then (optionally)
    all ranks receive every frame.  ``scenes`` entries are dicts of the pipeline's tensor arguments for one
    scene (leading batch dimension 1); all scenes of one call have the same view count."""

    def __init__(self, pipeline, rank: int = 0, world: int = 1):
        self.pipeline = pipeline
        self.rank, self.world = rank, world

    def plan(self, scenes: Sequence[dict], res: int) -> List[List[int]]:
        cfg = self.pipeline.config
        costs = [scene_cost(cfg, int(s["mask"].sum()), int(s["c2w"].shape[1]), res) for s in scenes]
        return assign_units(costs, self.world)

    def _frame_shape(self, n_views: int, res: int):
        return (n_views, res, res, frame_channels(self.pipeline.config))

    def render(self, scenes: Sequence[dict], res: int = 512, gather: bool = True, **kw):
        """Scenes sharded by LPT; returns [n_scenes, V, res, res, C] on every rank (gather) or
        (my scene ids, my frames)."""
        if not scenes:
            raise ValueError("no scenes")
        views = {int(s["c2w"].shape[1]) for s in scenes}
        if len(views) != 1:
            raise ValueError("all scenes of one call must have the same view count")
        mine = self.plan(scenes, res)[self.rank]
        frames = [self.pipeline(**scenes[i], resolution=res, **kw)[0] for i in mine]  # [V, H, W, C] each
        shape = self._frame_shape(views.pop(), res)
        local = (torch.stack(frames) if frames
                 else torch.empty((0,) + shape, dtype=torch.float32, device=self.pipeline.device))
        if not gather:
            return mine, local
        return gather_frames(local, mine, len(scenes))

    def render_views(self, scene: dict, res: int = 512, gather: bool = True, **kw):
        """One scene, its views split across ranks (shard_views); returns [V, res, res, C] on every rank
        (gather) or (my view range, my frames)."""
        n_views = int(scene["c2w"].shape[1])
        vr = shard_views(n_views, self.world)[self.rank]
        shape = self._frame_shape(n_views, res)[1:]
        if len(vr):
            sub = dict(scene)
            sub["c2w"] = scene["c2w"][:, vr.start:vr.stop].contiguous()
            sub["fov"] = scene["fov"][:, vr.start:vr.stop].contiguous()
            local = self.pipeline(**sub, resolution=res, **kw)[0]
        else:
            local = torch.empty((0,) + shape, dtype=torch.float32, device=self.pipeline.device)
        if not gather:
            return vr, local
        return gather_frames(local, list(vr), n_views)
