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

The data path is pipelined: loader threads decode and collate the next batches into
pinned host memory (texture kept in the dtype the file stores, widened on the device) while batch i renders, the
host-to-device copy runs on a side stream that the compute stream waits on, results come back on
another side stream, and writer threads encode and write the EXR/PNG files — the GPU only waits for
the HDF5 decode when that is slower than a batch.  RF_BATCH_INLINE=1 runs every step
inline on the main thread.
"""
from __future__ import annotations

import argparse
import glob
import os
import re
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

from infer import PRECISION, add_common_args, load_pipeline, save_views
from renderformer_amd.h5io import File
from renderformer_amd.parallel import assign_units, scene_cost


def natural_key(path: str):
    """natsort's default ordering for the file names used here (digit runs compare numerically)."""
    return [int(t) if t.isdigit() else t.lower() for t in re.split(r"(\d+)", path)]


def load_scene(path: str, padding_length=None, texture_dtype=torch.float32) -> dict:
    """`TriangleRenderH5Dataset.__getitem__` (batch_infer.py:27-58).  texture_dtype=None keeps the dtype the
    file stores (to_h5 writes fp16: half the host bytes; the pipelined path widens it to fp32 on the device,
    the same conversion the inline path does on the host)."""
    with File(path) as f:
        tri = torch.from_numpy(np.array(f["triangles"])).float()
        tex = torch.from_numpy(np.array(f["texture"]))
        if texture_dtype is not None:
            tex = tex.to(texture_dtype)
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


LOADERS = int(os.environ.get("RF_BATCH_LOADERS", "3"))  # batches decoded ahead (threads)
WRITERS = 4  # image encode/write threads
DEPTH = max(1, int(os.environ.get("RF_BATCH_DEPTH", "2")))  # batches in flight behind the one being issued


def _one_omp_thread():
    """Pool-thread initializer: the loader / writer threads' own torch CPU ops run single-threaded.  Every thread that
    enters an OpenMP region gets its own team of workers (libgomp), which spin after each region: 3 loaders + 4 writers
    on a 16-thread host made ~100 extra threads that burned ~0.1 CPU-s per frame (profiles/r6_host_budget.txt),
    the cores the HDF5 inflate pool needs."""
    torch.set_num_threads(1)


class StageTimes:
    """Per-stage host time of the data path (RF_BATCH_PROFILE=1; tools/batch_e2e.py): seconds summed over the
    threads that ran each stage, plus the main thread's wall time blocked in each wait."""

    def __init__(self):
        import threading
        self.on = os.environ.get("RF_BATCH_PROFILE", "0") != "0"
        self.t = {}
        self.n = {}
        self._lock = threading.Lock()

    def add(self, name, dt):
        if self.on:
            with self._lock:
                self.t[name] = self.t.get(name, 0.0) + dt
                self.n[name] = self.n.get(name, 0) + 1

    def timed(self, name, fn, *a, **k):
        if not self.on:
            return fn(*a, **k)
        t0, c0 = time.perf_counter(), time.thread_time()
        try:
            return fn(*a, **k)
        finally:
            self.add(name, time.perf_counter() - t0)
            self.add("cpu: " + name, time.thread_time() - c0)  # this thread's CPU seconds in the stage

    def summary(self):
        return {k: {"s": round(v, 4), "calls": self.n[k]} for k, v in sorted(self.t.items())}

    def host_budget(self, frames: int, wall: float, proc_cpu: float) -> dict:
        """CPU seconds per frame of this rank: the whole process (every thread: loader, HDF5 chunk decode pool, main,
        writers, torch's own), and the main items — what a rank needs of the node's cores at a given frame rate."""
        g = lambda k: self.t.get(k, 0.0) / max(frames, 1)  # noqa: E731
        per = {"process_cpu_s": proc_cpu / max(frames, 1), "hdf5_chunk_decode_cpu_s": g("cpu: h5 chunk decode"),
               "exr_write_cpu_s": g("cpu: write: EXR"), "png_write_cpu_s": g("cpu: write: PNG"),
               "render_issue_cpu_s": g("cpu: main: render issue (plan + launches)")}
        fps = frames / wall if wall > 0 else 0.0
        return {"frames": frames, "wall_s": round(wall, 4), "frames_per_s": round(fps, 2),
                "per_frame": {k: round(v, 5) for k, v in per.items()},
                "cores_busy_at_this_rate": round(per["process_cpu_s"] * fps, 2)}


STAGES = StageTimes()


class ThreadCpu:
    """Profiling only (RF_BATCH_PROFILE): CPU seconds of every OS thread of this process over the data path, from
    /proc/self/task/<tid>/stat sampled every 0.2 s (a thread that exits between samples loses at most one period),
    labelled by the Python thread's name (pool suffix dropped) or, for threads Python did not start (torch's
    OpenMP workers, the HIP runtime's), by the kernel's comm name -- where the host budget's cores go."""

    def __init__(self):
        import threading
        self._tick = os.sysconf("SC_CLK_TCK")
        self._first, self._last, self._label, self._wchan = {}, {}, {}, {}
        self._stop = threading.Event()
        self._started = False
        self._sample()  # threads alive now count from here; threads born later from zero
        self._started = True
        self._t = threading.Thread(target=self._run, name="rf_cpu_sampler", daemon=True)
        self._t.start()

    def _sample(self):
        import re
        import threading
        names = {t.native_id: re.sub(r"_\d+$", "", t.name) for t in threading.enumerate()}
        try:
            tids = os.listdir("/proc/self/task")
        except OSError:
            return
        for tid in tids:
            try:
                with open(f"/proc/self/task/{tid}/stat") as f:
                    st = f.read()
            except OSError:
                continue
            comm = st[st.index("(") + 1:st.rindex(")")]
            fields = st[st.rindex(")") + 2:].split()
            cpu = (int(fields[11]) + int(fields[12])) / self._tick  # utime + stime
            t = int(tid)
            self._first.setdefault(t, cpu if not self._started else 0.0)
            self._last[t] = cpu
            self._label.setdefault(t, names.get(t) or "os:" + comm)
            if self._label[t].startswith("os:"):  # where a foreign thread sleeps ("0": running), most frequent wins
                try:
                    with open(f"/proc/self/task/{tid}/wchan") as f:
                        w = f.read().strip() or "0"
                except OSError:
                    w = "?"
                c = self._wchan.setdefault(t, {})
                c[w] = c.get(w, 0) + 1

    def _run(self):
        while not self._stop.wait(0.2):
            self._sample()

    def stop(self) -> dict:
        self._stop.set()
        self._t.join()
        self._sample()
        out = {}
        for t, c in self._last.items():
            lab = self._label[t]
            if t in self._wchan:
                lab += "@" + max(self._wchan[t].items(), key=lambda x: x[1])[0]
            n, s = out.get(lab, (0, 0.0))
            out[lab] = (n + 1, s + c - self._first[t])
        return {k: {"threads": n, "cpu_s": round(s, 3)} for k, (n, s) in sorted(out.items(), key=lambda x: -x[1][1])}


def _load_batch(files, idx, padding_length, pin):
    if pin:
        return _load_batch_pinned(files, idx, padding_length)
    items = [STAGES.timed("load: HDF5 read + inflate", load_scene, files[i], padding_length, torch.float32)
             for i in idx]
    host = STAGES.timed("load: collate", collate, items)
    return items, host


def _load_batch_pinned(files, idx, padding_length, pinned: bool = True):
    """The batch's tensors allocated once in pinned host memory (torch's caching host allocator) with every scene
    decoded straight into its slot (h5io read(out=)): no per-scene array, no collate stack and no pin_memory()
    copy -- those two full copies of the ~150-300 MB texture were a third of a scene's host time.  Same result as
    collate(load_scene(...)) + pin_memory(): the file's texture dtype, zero padding rows, padded mask False."""
    t0 = time.perf_counter()
    fs = [File(files[i]) for i in idx]
    try:
        ns = [f["triangles"].shape[0] for f in fs]
        if padding_length is not None:
            for i, n in zip(idx, ns):
                if padding_length < n:
                    raise ValueError(f"{files[i]}: {n} triangles exceed --padding_length {padding_length}")
            N = padding_length
        else:
            if len(set(ns)) > 1:
                raise ValueError("scenes in one batch differ in shape: pass --padding_length (as the reference requires)")
            N = ns[0]
        views = {f["c2w"].shape[0] for f in fs}
        if len(views) > 1:
            raise ValueError("scenes in one batch differ in shape: pass --padding_length (as the reference requires)")
        B, V = len(fs), views.pop()
        tex_ds = [f["texture"] for f in fs]
        tdt = {torch.from_numpy(np.empty(0, dtype=d.dtype)).dtype for d in tex_ds}
        if len(tdt) > 1:
            raise ValueError("scenes in one batch store textures of different dtypes")
        pin = dict(pin_memory=pinned)  # (pinned=False: the same decode into pageable memory, for CPU tests)
        host = {"triangles": torch.zeros(B, N, 3, 3, dtype=torch.float32, **pin),
                "texture": torch.empty(B, N, *tex_ds[0].shape[1:], dtype=tdt.pop(), **pin),
                "mask": torch.zeros(B, N, dtype=torch.bool, **pin),
                "c2w": torch.empty(B, V, 4, 4, dtype=torch.float32, **pin),
                "fov": torch.empty(B, V, dtype=torch.float32, **pin),
                "vn": torch.zeros(B, N, 3, 3, dtype=torch.float32, **pin)}
        items = []
        for b, (f, n) in enumerate(zip(fs, ns)):
            tex = host["texture"][b]
            tex_ds[b].read(out=tex[:n].numpy())
            if n < N:
                tex[n:].zero_()
            host["triangles"][b, :n] = torch.from_numpy(np.array(f["triangles"])).float()
            host["vn"][b, :n] = torch.from_numpy(np.array(f["vn"])).float()
            host["c2w"][b] = torch.from_numpy(np.array(f["c2w"]).astype(np.float32))
            host["fov"][b] = torch.from_numpy(np.array(f["fov"]).astype(np.float32).reshape(V))
            host["mask"][b, :n] = True
            items.append({"file_path": files[idx[b]]})
    finally:
        for f in fs:
            f.close()
    STAGES.add("load: HDF5 read + inflate into pinned", time.perf_counter() - t0)
    return items, host


_COPY_STREAMS = {}


def _runs_beside(s, compute) -> bool:
    """Does work on stream `s` start while `compute` is busy?  HIP maps streams onto a few hardware queues
    (GPU_MAX_HW_QUEUES, 4 here) round robin; two streams on one queue run in submission order, so a copy stream that
    shares the compute stream's queue serializes every H2D with the frames' kernels.  Probe: a ~10 ms spin on `compute`,
    then an event on the idle `s`, which completes at once unless it is queued behind the spin."""
    with torch.cuda.stream(compute):
        torch.cuda._sleep(int(2e7))
    ev = torch.cuda.Event()
    ev.record(s)
    t0 = time.perf_counter()
    ok = False
    while time.perf_counter() - t0 < 0.004:
        if ev.query():
            ok = True
            break
    compute.synchronize()
    return ok


def _copy_streams(dev):
    """The side streams of the H2D / D2H copies, made once per (device, compute stream): pool streams that the probe
    finds on a hardware queue of their own (profiles/r6_batch_e2e.txt: a copy stream on the compute stream's queue
    cost 10-15 % end to end, in every other batch_infer call as the pool's round robin came back to that queue).
    RF_BATCH_COPY_STREAMS=perpass: two new pool streams per call, unprobed (the round-5 behaviour)."""
    if os.environ.get("RF_BATCH_COPY_STREAMS", "probed") == "perpass":
        return torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    compute = torch.cuda.current_stream(dev)
    key = (str(dev), compute.cuda_stream)
    if key not in _COPY_STREAMS:
        got = []
        for _ in range(16):  # the pool hands its streams out round robin over the queues
            s = torch.cuda.Stream(device=dev)
            if _runs_beside(s, compute):
                got.append(s)
                if len(got) == 2:
                    break
        while len(got) < 2:  # no free queue found: keep whatever the pool gives (correct, only slower)
            got.append(torch.cuda.Stream(device=dev))
        _COPY_STREAMS[key] = tuple(got)
    return _COPY_STREAMS[key]


def render_batches(pipeline, files, batches, args, pipelined=True):
    """Yield (items, hdr images on the host) per batch, in order.  Pipelined: loader thread -> pinned batch
    -> side-stream H2D -> render on the current stream -> side-stream D2H into pinned memory; batch i is
    yielded (and its files written by the caller) while batch i+1 renders and batch i+2 loads."""
    dev = pipeline.device
    kw = dict(resolution=args.resolution, torch_dtype=PRECISION[args.precision])

    model = getattr(pipeline, "model", None)
    resolve = getattr(pipeline, "resolve", None)

    def render(batch, host=None):
        if host is not None and hasattr(model, "plan_hint"):  # a new scene's plan from the host mask: no read-back
            model.plan_hint(batch["mask"], host["mask"].numpy())
        tex = batch["texture"]
        if tex.dtype != torch.float32:  # the file's dtype, widened on the device like the inline path's host cast
            tex = tex.float()
        return pipeline(triangles=batch["triangles"], texture=tex, mask=batch["mask"], vn=batch["vn"],
                        c2w=batch["c2w"], fov=batch["fov"].unsqueeze(-1), **kw)

    if not pipelined or dev.type != "cuda":
        for idx in batches:
            items, host = _load_batch(files, idx, args.padding_length, False)
            imgs = render({k: v.to(dev) for k, v in host.items()}, host)
            if resolve is not None:
                resolve(imgs)
            yield items, imgs.cpu()
        return
    # HDF5 decode (zlib releases the GIL) runs LOADERS batches ahead on a thread pool, consumed in order
    pool = ThreadPoolExecutor(max_workers=LOADERS, thread_name_prefix="rf_loader", initializer=_one_omp_thread)
    ahead = [pool.submit(_load_batch, files, idx, args.padding_length, True) for idx in batches[:LOADERS]]
    nxt_batch = len(ahead)

    class _Loaded:
        def get(self):
            nonlocal nxt_batch
            if not ahead:
                pool.shutdown(wait=False)
                return None
            fut = ahead.pop(0)
            if nxt_batch < len(batches):
                ahead.append(pool.submit(_load_batch, files, batches[nxt_batch], args.padding_length, True))
                nxt_batch += 1
            try:
                return STAGES.timed("main: wait for loader", fut.result)
            except BaseException as e:  # surfaced on the main thread
                return e

    loaded = _Loaded()
    h2d, d2h = _copy_streams(dev)
    compute = torch.cuda.current_stream(dev)
    # (items, pinned host images, their copy event, pinned inputs, device images) of the batches in flight: batch i is
    # handed out once batch i + DEPTH is issued, so a late loader or a slow issue does not drain the GPU's queue
    pending = []

    def upload():
        """The next loaded batch (waiting for the loader if it is late) copied to the device on the H2D stream."""
        got = loaded.get()
        if isinstance(got, BaseException):
            raise got
        if got is None:
            return None
        items, host = got
        t_h = time.perf_counter()
        with torch.cuda.stream(h2d):
            batch = {k: v.to(dev, non_blocking=True) for k, v in host.items()}
            copied_in = torch.cuda.Event()
            copied_in.record(h2d)
        STAGES.add("main: H2D issue", time.perf_counter() - t_h)
        return items, host, batch, copied_in

    # batch i + 1's H2D is issued right after batch i's kernels, so the ~150-300 MB texture copy runs under batch i's
    # frame instead of in front of batch i + 1's (profiles/r6_batch_e2e.txt: the GPU idled behind the copy otherwise)
    staged = upload()
    while True:
        nxt = None
        cur, staged = staged, None
        if cur is not None:
            items, host, batch, copied_in = cur
            compute.wait_event(copied_in)
            for v in batch.values():  # allocated on the copy stream, used on the compute stream
                v.record_stream(compute)
            imgs = STAGES.timed("main: render issue (plan + launches)", render, batch, host)
            # the result goes back on its own stream right behind this batch, not behind the next one
            d2h.wait_stream(compute)
            with torch.cuda.stream(d2h):
                out = torch.empty(imgs.shape, dtype=imgs.dtype, pin_memory=True)
                out.copy_(imgs, non_blocking=True)
                copied = torch.cuda.Event()
                copied.record(d2h)
            imgs.record_stream(d2h)
            nxt = (items, out, copied, host, imgs)  # `host` (pinned inputs) lives until this batch is yielded
            staged = upload()
        if nxt is not None:
            pending.append(nxt)
        while pending and (len(pending) > DEPTH or nxt is None):  # batch i is handed out while i+1.. render
            p_items, p_out, p_copied, _, p_imgs = pending.pop(0)
            STAGES.timed("main: wait for frame + D2H", p_copied.synchronize)
            # the frame is complete: its fp16 range check reads a host word (no wait); a frame that overflowed is
            # rendered again in place, and copied back again
            if resolve is not None and STAGES.timed("main: range check", resolve, p_imgs):
                p_out.copy_(p_imgs)
            t_y = time.perf_counter()
            yield p_items, p_out
            STAGES.add("main: consumer (writer submission)", time.perf_counter() - t_y)
        if nxt is None:
            return


def main(argv=None, pipeline=None):
    """The CLI.  `pipeline`: an already-built RenderFormerRenderingPipeline for the same model flags (tools/batch_e2e.py
    times the data path apart from the model build)."""
    parser = argparse.ArgumentParser(description="Batch inference using triangle radiosity transformer model (MI355X)")
    parser.add_argument("--h5_folder", type=str, required=True)
    parser.add_argument("--batch_size", type=int, default=8)
    parser.add_argument("--padding_length", type=int, default=None)
    parser.add_argument("--num_workers", type=int, default=0,
                        help="accepted for compatibility (loading always runs in one background thread)")
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
    t_build = time.perf_counter()
    if pipeline is None:
        pipeline = load_pipeline(args)
    STAGES.add("main: model build (load_pipeline)", time.perf_counter() - t_build)
    t_loop = time.perf_counter()
    cpu0 = time.process_time()  # every thread of this process (loader, chunk decode pool, main, writers)
    threads = None
    if STAGES.on:
        from renderformer_amd import h5io
        h5io.CPU_HOOK = lambda dt: STAGES.add("cpu: h5 chunk decode", dt)
        threads = ThreadCpu()
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
    batches = [mine[b0:b0 + args.batch_size] for b0 in range(0, len(mine), args.batch_size)]
    n_frames = 0
    inline = os.environ.get("RF_BATCH_INLINE", "0") != "0"
    writers = None if inline else ThreadPoolExecutor(max_workers=WRITERS, thread_name_prefix="rf_writer",
                                                    initializer=_one_omp_thread)
    pending = []
    for items, imgs in render_batches(pipeline, files, batches, args, pipelined=not inline):
        for i, it in enumerate(items):
            base = os.path.splitext(os.path.basename(it["file_path"]))[0]
            if writers is None:
                save_views(imgs[i], output_dir, base, STAGES)
            else:  # EXR/PNG encode + write off the render loop (zlib releases the GIL)
                pending.append(writers.submit(save_views, imgs[i], output_dir, base, STAGES))
            n_frames += imgs.shape[1]
    if writers is not None:
        for f in pending:
            STAGES.timed("main: wait for writers", f.result)  # re-raises a writer's error
        writers.shutdown()
    wall = time.perf_counter() - t_loop
    STAGES.add("main: data path wall (first load -> last file)", wall)
    print(f"Output saved to: {output_dir} ({n_frames} frames on rank {rank}/{world})")
    if STAGES.on:
        import json
        from renderformer_amd import h5io
        h5io.CPU_HOOK = None
        print("stage times:", json.dumps(STAGES.summary()), flush=True)
        print("host budget:", json.dumps(STAGES.host_budget(n_frames, wall, time.process_time() - cpu0)), flush=True)
        print("thread cpu:", json.dumps(threads.stop()), flush=True)
    if args.save_video:
        print("video.mp4 not written: no mp4 encoder in this environment (frames are saved as PNG)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
