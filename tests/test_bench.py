"""bench.py's launcher contract (CPU) and its multi-rank path on one GPU (gloo, every rank on cuda:0)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def test_gpus_must_match_world_size(monkeypatch, capsys):
    import bench
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    assert bench.main() == 2  # refused before any GPU call
    assert "WORLD_SIZE=1" in capsys.readouterr().err


def test_gpus_n_starts_n_ranks(monkeypatch):
    """Without a torch.distributed.run environment, --gpus N starts one process per GPU as a child."""
    import bench
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    seen = {}
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd: seen.setdefault("cmd", cmd) and 0)
    assert bench.main() == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-4:] == ["--gpus", "4", "--steps", "3"]


def _bench(tmp_path, tag, gpus, extra):
    dump = str(tmp_path / f"{tag}.npy")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(gpus), "--steps", "1", "--warmup", "0",
           "--no-cpu-baseline", "--config", "base", "--res", "256", "--dump", dump] + extra
    if gpus > 1:
        cmd += ["--backend", "gloo", "--same-device"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line), np.load(dump)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_two_ranks_match_one(tmp_path):
    """The same bench workload on 1 and 2 ranks (2 processes on the one GPU of the box, gloo all_gather) gives
    bit-identical gathered frames: 64-scene-style LPT sharding (3 example scenes), and the views of
    one scene split over ranks (c5: stage 2 + DPT per view, --view-chunk 1, so a view runs the same launches
    whatever the split)."""
    r1, f1 = _bench(tmp_path, "c4_1", 1, ["--workload", "c4", "--scenes", "3"])
    r2, f2 = _bench(tmp_path, "c4_2", 2, ["--workload", "c4", "--scenes", "3"])
    assert r1["n_gpus"] == 1 and r2["n_gpus"] == 2 and r2["scaling"] == "strong"
    assert f1.shape == (3, 256, 256, 3) and f2.shape == f1.shape
    assert np.array_equal(f1, f2)
    v1 = _bench(tmp_path, "c5_1", 1, ["--workload", "c5", "--views", "3", "--tris", "800"])[1]
    v2 = _bench(tmp_path, "c5_2", 2, ["--workload", "c5", "--views", "3", "--tris", "800"])[1]
    assert v1.shape == (3, 256, 256, 3) and v2.shape == v1.shape
    assert np.array_equal(v1, v2)
