"""CPU multi-process test (gloo, world size 2) of the image-tile split + gather path (cudaraytracer_amd.parallel):
each rank renders its block-cyclic row bands with the CPU oracle, the bands are gathered to rank 0 over
torch.distributed and reassembled, and the result must equal the single-process frame bit for bit."""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, band_rows: int, out_path: str) -> None:
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from cudaraytracer_amd import parallel, scenes
    from cudaraytracer_amd.renderer import band_rows_of
    from oracle import py_oracle as po

    parallel.init_process_group("gloo")
    cfg = scenes.CONFIGS["c2"].scaled(96, 72, 2)
    sc = po.OracleScene(scenes.builtin(cfg.scene))
    rows = band_rows_of(cfg.height, band_rows, world, rank)
    st = po.init_states(cfg.width, cfg.height)
    img, _, _ = po.render(sc, cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st, threads=1)
    local = torch.from_numpy(img[rows].astype(np.int64).reshape(-1))  # this rank's bands only
    full = parallel.gather_bands(local, cfg.width, cfg.height, band_rows)
    if rank == 0:
        np.save(out_path, full.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _pipelined_worker(rank: int, world: int, port: int, band_rows: int, out_path: str, height: int = 37) -> None:
    """BandGather as bench.py drives it: frame k's gather is started, frame k + 1 is "rendered" (the local
    buffer overwritten) before frame k is finished; rank 0 keeps every finished frame."""
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from cudaraytracer_amd import parallel
    from cudaraytracer_amd.renderer import band_rows_of

    parallel.init_process_group("gloo")
    width = 5
    rows = torch.tensor(band_rows_of(height, band_rows, world, rank), dtype=torch.int64)
    local = torch.empty(len(rows) * width, dtype=torch.int64)
    g = parallel.BandGather(width, height, band_rows)
    frames = []
    for k in range(4):
        local.copy_((rows[:, None] * width + torch.arange(width) + 1000 * k).reshape(-1))  # frame k
        if k:
            prev = g.finish()
            if rank == 0:
                frames.append(prev.clone())
        g.start(local)
    last = g.finish()
    if rank == 0:
        frames.append(last.clone())
        np.save(out_path, torch.stack(frames).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world, band_rows, height", [(2, 16, 37), (3, 4, 37), (8, 16, 4320)])
def test_pipelined_band_gather_keeps_frames_apart(tmp_path, world, band_rows, height):
    """World size 8 with BASELINE config 4's 4320 rows in 16-row bands: 270 bands, so the last
    round is ragged (ranks 0-5 hold 34 bands, 6 and 7 hold 33) — the 8-GPU scaling run's C4 gather."""
    out = str(tmp_path / "frames.npy")
    mp.start_processes(_pipelined_worker, args=(world, _free_port(), band_rows, out, height), nprocs=world,
                       start_method="spawn")
    frames = np.load(out)
    base = np.arange(height * 5).reshape(height, 5)
    assert frames.shape == (4, height, 5)
    for k in range(4):
        np.testing.assert_array_equal(frames[k], base + 1000 * k)


@pytest.mark.parametrize("world, band_rows", [(2, 16), (2, 5), (3, 16)])
def test_gather_bands_reassembles_the_frame(tmp_path, world, band_rows):
    sys.path.insert(0, ROOT)
    from cudaraytracer_amd import scenes
    from oracle import py_oracle as po

    out = str(tmp_path / "full.npy")
    mp.start_processes(_worker, args=(world, _free_port(), band_rows, out), nprocs=world, start_method="spawn")
    cfg = scenes.CONFIGS["c2"].scaled(96, 72, 2)
    st = po.init_states(cfg.width, cfg.height)
    ref, _, _ = po.render(po.OracleScene(scenes.builtin(cfg.scene)), cfg.width, cfg.height, cfg.spp, cfg.depth,
                          cfg.inputs(), st, threads=1)
    np.testing.assert_array_equal(np.load(out).astype(np.uint32), ref)


def test_band_rows_partition_the_image():
    sys.path.insert(0, ROOT)
    from cudaraytracer_amd.renderer import band_rows_of

    for h, b, n in [(1080, 16, 8), (37, 16, 3), (4320, 16, 8), (7, 16, 4)]:
        rows = sorted(r for k in range(n) for r in band_rows_of(h, b, n, k))
        assert rows == list(range(h))


@pytest.mark.parametrize("height, band_rows, world", [(72, 16, 2), (72, 5, 3), (37, 16, 8), (128, 16, 8), (4320, 16, 8),
                                                      (17, 4, 1), (3, 16, 4)])
def test_unshuffle_matches_row_index_reassembly(height, band_rows, world):
    """The strided unshuffle puts every rank's local rows at the global rows band_rows_of assigns them."""
    sys.path.insert(0, ROOT)
    from cudaraytracer_amd import parallel
    from cudaraytracer_amd.renderer import band_rows_of

    width = 7
    frame = torch.arange(height * width, dtype=torch.int64).view(height, width)
    counts = [len(band_rows_of(height, band_rows, world, r)) for r in range(world)]
    recv = []
    for r in range(world):
        rows = band_rows_of(height, band_rows, world, r)
        buf = torch.full((max(counts) * width,), -1, dtype=torch.int64)
        if rows:
            buf[: len(rows) * width] = frame[rows].reshape(-1)
        recv.append(buf)
    full = torch.full((height, width), -2, dtype=torch.int64)
    parallel.unshuffle_into(full, recv, height, width, band_rows)
    assert torch.equal(full, frame)
