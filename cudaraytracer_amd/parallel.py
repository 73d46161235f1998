"""Image-tile split across ranks + gather of the per-rank framebuffers.

One process per GPU.  Rank r renders the block-cyclic row bands b ≡ r (mod N) of the image into a
contiguous local buffer (rt_tiling in include/rt_hip.h; RNG seeds and camera use the GLOBAL pixel index,
so the N-rank image is bit-identical to the 1-rank image).  The only exchange is one gather of the local
RGBA8 buffers to the destination rank over torch.distributed (RCCL over xGMI on MI355X, gloo on CPU),
followed by the inverse row permutation.  The reference has no multi-GPU path; this is the north star's
"image optionally tiled across the 8 GPUs of one node with an RCCL gather".
"""
from __future__ import annotations

import functools
import os

import torch
import torch.distributed as dist

from .renderer import band_rows_of

DEFAULT_BAND_ROWS = 16  # one workgroup tile row (render.hip: 16×16 pixels per workgroup)


def env_rank() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment (1 process = rank 0)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def init_process_group(backend: str) -> None:
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        dist.init_process_group(backend=backend)


@functools.lru_cache(maxsize=64)
def local_row_counts(height: int, band_rows: int, world: int) -> list[int]:
    return [len(band_rows_of(height, band_rows, world, r)) for r in range(world)]


_BUFFERS: dict = {}


def _buffers(key, world: int, rank: int, dst: int, max_rows: int, width: int, height: int, dtype, dev):
    """Send / receive / frame buffers of one gather shape, allocated once (the bench gathers every step)."""
    b = _BUFFERS.get(key)
    if b is None:
        if len(_BUFFERS) > 16:
            _BUFFERS.clear()
        send = torch.zeros(max_rows * width, dtype=dtype, device=dev)
        recv = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
        full = torch.empty(height, width, dtype=dtype, device=dev) if rank == dst else None
        b = _BUFFERS[key] = (send, recv, full)
    return b


def unshuffle_into(full: torch.Tensor, recv: list, height: int, width: int, band_rows: int) -> None:
    """Rank r's local rows are the bands r, r + N, r + 2N, ... of the frame: every complete round of N bands
    is one strided copy per rank, the ragged last round one small copy per rank."""
    world = len(recv)
    rnd = band_rows * world
    k = height // rnd
    if k:
        full4 = full[: k * rnd].view(k, world, band_rows, width)
        for r in range(world):
            full4[:, r].copy_(recv[r][: k * band_rows * width].view(k, band_rows, width))
    base = k * band_rows * width
    for r in range(world):
        start = k * rnd + r * band_rows
        if start >= height:
            break
        n = min(band_rows, height - start)
        full[start:start + n].copy_(recv[r][base: base + n * width].view(n, width))


def gather_bands(local: torch.Tensor, width: int, height: int, band_rows: int, dst: int = 0,
                 group=None, reuse: bool = False) -> torch.Tensor | None:
    """Gather every rank's (local_rows·W) framebuffer to `dst` and return the (H, W) image there.  The result
    is a fresh tensor unless `reuse` is set: then it is a module-owned buffer that the next gather of the same
    shape overwrites (the bench, which gathers every step and keeps no frame).  With the gloo backend (CPU
    tests, single-GPU rehearsals) device buffers are staged through host memory."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = local_row_counts(height, band_rows, world)
    max_rows = max(counts)
    via_host = local.is_cuda and dist.get_backend(group) == "gloo"
    dev = torch.device("cpu") if via_host else local.device
    # keyed by the group object itself (held in the key, so a destroyed group's id cannot be reused by another)
    key = (group, world, rank, dst, max_rows, width, height, band_rows, local.dtype, str(dev))
    send, recv, full = _buffers(key, world, rank, dst, max_rows, width, height, local.dtype, dev)
    send[: local.numel()].copy_(local.reshape(-1))
    dist.gather(send, recv, dst=dst, group=group)
    if rank != dst:
        return None
    unshuffle_into(full, recv, height, width, band_rows)
    if via_host:
        return full.to(local.device)
    return full if reuse else full.clone()


class BandGather:
    """Pipelined per-frame gather (the bench's multi-rank step): start(local) enqueues frame k's gather on the
    collective's own stream and returns at once, so the caller's next render overlaps it; the next start (or
    finish) makes the caller's stream wait for frame k's gather and unshuffles it on `dst`.  The send buffer is
    refilled only after that wait, so a gather never reads a frame being rendered.  Device tensors under gloo
    (one-GPU rehearsals) are gathered synchronously inside start; CPU tensors under gloo take the pipelined
    path (tests/test_distributed.py)."""

    def __init__(self, width: int, height: int, band_rows: int, dst: int = 0, group=None):
        self.width, self.height, self.band_rows, self.dst, self.group = width, height, band_rows, dst, group
        self.work = None
        self.bufs = None

    def start(self, local: torch.Tensor) -> None:
        self.finish()
        group = self.group
        if local.is_cuda and dist.get_backend(group) == "gloo":  # device buffers staged through the host
            self.result = gather_bands(local, self.width, self.height, self.band_rows, self.dst, group, reuse=True)
            return
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        counts = local_row_counts(self.height, self.band_rows, world)
        key = (group, world, rank, self.dst, max(counts), self.width, self.height, self.band_rows, local.dtype,
               str(local.device), "pipelined")
        self.bufs = _buffers(key, world, rank, self.dst, max(counts), self.width, self.height, local.dtype,
                             local.device)
        send, recv, _ = self.bufs
        send[: local.numel()].copy_(local.reshape(-1))
        self.work = dist.gather(send, recv, dst=self.dst, group=group, async_op=True)

    def finish(self) -> torch.Tensor | None:
        """The last started frame's (H, W) image on dst (None elsewhere); the caller's stream waits for it."""
        if self.work is not None:
            self.work.wait()
            self.work = None
            _, recv, full = self.bufs
            self.result = None
            if dist.get_rank(self.group) == self.dst:
                unshuffle_into(full, recv, self.height, self.width, self.band_rows)
                self.result = full
        return getattr(self, "result", None)
