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


@functools.lru_cache(maxsize=64)
def _rows_index(height: int, band_rows: int, world: int, rank: int, device: str) -> torch.Tensor:
    return torch.tensor(band_rows_of(height, band_rows, world, rank), dtype=torch.long, device=device)


def gather_bands(local: torch.Tensor, width: int, height: int, band_rows: int, dst: int = 0,
                 group=None) -> torch.Tensor | None:
    """Gather every rank's (local_rows·W) framebuffer to `dst` and return the (H, W) image there.  With
    the gloo backend (CPU tests, single-GPU rehearsals) device buffers are staged through host memory."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = local_row_counts(height, band_rows, world)
    max_rows = max(counts)
    via_host = local.is_cuda and dist.get_backend(group) == "gloo"
    dev = torch.device("cpu") if via_host else local.device
    send = torch.zeros(max_rows * width, dtype=local.dtype, device=dev)
    send[: local.numel()] = local.reshape(-1).to(dev)
    recv = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, recv, dst=dst, group=group)
    if rank != dst:
        return None
    full = torch.empty(height, width, dtype=local.dtype, device=dev)
    for r in range(world):
        full.index_copy_(0, _rows_index(height, band_rows, world, r, str(dev)), recv[r][: counts[r] * width].view(counts[r], width))
    return full.to(local.device) if via_host else full
