"""CPU tests of bench.py's multi-rank launch (no GPU): `--gpus N` without a launcher starts its own N ranks
(a child torch.distributed.run), refuses to run when fewer than N GPUs are visible, and the launched ranks
see world size N (rehearsed with `--dry-run`: gloo ranks gathering synthetic bands)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


@pytest.mark.parametrize("gpus, config", [(2, "c2"), (3, "c4"), (8, "c4")])
def test_self_launch_spawns_n_ranks(gpus, config):
    p = _bench("--gpus", str(gpus), "--config", config, "--dry-run")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 prints one line
    assert lines[0]["world_size"] == gpus and lines[0]["frame_ok"] is True


@pytest.mark.parametrize("gpus", [2, 3, 8])
def test_default_line_carries_config4_block(gpus):
    """the driver's default `bench.py --gpus N` (config 2) also measures BASELINE config 4 (the
    7680x4320 frame split over the N ranks + the gather): the rehearsed launch carries other_configs.c4."""
    p = _bench("--gpus", str(gpus), "--dry-run")
    assert p.returncode == 0, p.stderr[-2000:]
    line = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")][0]
    c4 = line["other_configs"]["c4"]
    assert c4["frame_ok"] is True and c4["height"] == 4320 and c4["scaling"] == "strong"
    assert line["world_size"] == gpus and line["frame_ok"] is True


def test_fewer_gpus_than_requested_fails_loudly():
    """The driver's `python bench.py --gpus N` must never print a 1-GPU line for N > 1 (this container has no GPU)."""
    p = _bench("--gpus", "2", "--steps", "1", "--warmup", "0", timeout=120)
    assert p.returncode != 0
    assert "needs 2 visible GPUs" in p.stderr
    assert not any(ln.startswith("{") for ln in p.stdout.splitlines())


def test_launched_rank_checks_world_size(monkeypatch):
    """Under a launcher whose WORLD_SIZE disagrees with --gpus, a rank exits instead of reporting a wrong N."""
    sys.path.insert(0, ROOT)
    import bench

    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("LOCAL_RANK", "0")
    with pytest.raises(SystemExit, match="WORLD_SIZE=1 but --gpus 2"):
        bench.dry_run(bench.parse_args(["--gpus", "2", "--dry-run"]))


def test_configs_accepted():
    sys.path.insert(0, ROOT)
    import bench

    for c in ("c2", "c3", "c4", "c5"):
        assert bench.parse_args(["--config", c]).config == c
        assert c in bench.METRICS and c in bench.DATA
