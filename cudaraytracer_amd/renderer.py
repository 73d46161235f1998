"""Host-side mirror of the reference's render caller (CudaLayer, Cuda/CudaLayer.cpp) over the C ABI.

`Renderer` owns the device framebuffer and RNG-state buffers (InitCudaBuffers, CudaLayer.cpp:68-74), seeds
the RNG (RunCudaInit → RenderInit, CudaLayer.cpp:93-101), holds the device scene (GenerateWorld,
CudaLayer.cpp:103-256) and renders frames (RunCudaUpdate → LaunchKernel, CudaLayer.cpp:372-375).  Device
memory is allocated through torch (plumbing only); every compute step is a librt_hip.so call.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import abi
from ._lib import RTError, check, lib
from .scenes import Scene


class DeviceScene:
    """rt_scene handle (device-resident BVH + primitive + material tables)."""

    def __init__(self, scene: Scene | None = None, reference_graph: int | None = None):
        L = lib()
        self.handle = C.c_void_p()
        self.scene = scene
        if reference_graph is not None:
            check(L.rt_scene_from_reference_graph(C.c_void_p(reference_graph), C.byref(self.handle)),
                  "rt_scene_from_reference_graph")
        else:
            self._desc = scene.desc()
            check(L.rt_scene_create(C.byref(self._desc), C.byref(self.handle)), "rt_scene_create")

    def info(self) -> abi.SceneInfo:
        out = abi.SceneInfo()
        check(lib().rt_scene_get_info(self.handle, C.byref(out)), "rt_scene_get_info")
        return out

    def update_materials(self, materials) -> None:
        check(lib().rt_scene_update_materials(self.handle, C.cast(materials, C.POINTER(abi.MaterialDesc)),
                                              len(materials)), "rt_scene_update_materials")

    def close(self) -> None:
        if self.handle:
            lib().rt_scene_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def band_rows_of(height: int, band_rows: int, num_ranks: int, rank: int) -> list[int]:
    """Global rows owned by `rank` under block-cyclic row bands (rt_tiling, include/rt_hip.h)."""
    rows = []
    b = rank
    while b * band_rows < height:
        rows.extend(range(b * band_rows, min(height, (b + 1) * band_rows)))
        b += num_ranks
    return rows


class Renderer:
    """One rank's share of a W×H image (all of it when num_ranks = 1)."""

    def __init__(self, width: int, height: int, device: int | str = 0, band_rows: int | None = None,
                 num_ranks: int = 1, rank: int = 0, rng: str = "xorwow", state_layout: str = "curand"):
        """rng = "xorwow": the reference's per-pixel cuRAND XORWOW state (parity mode); "philox": stateless
        per-pixel Philox4x32-10 streams (RT_FLAG_RNG_PHILOX, perf mode, no RNG bytes in HBM).
        state_layout (XORWOW): "curand" = the reference's 48-byte curandState per pixel; "soa" = the same
        states as six uint32 planes (RT_FLAG_STATE_SOA, 24 bytes per pixel)."""
        if rng not in ("xorwow", "philox"):
            raise ValueError(f"rng must be 'xorwow' or 'philox', not {rng!r}")
        if state_layout not in ("curand", "soa"):
            raise ValueError(f"state_layout must be 'curand' or 'soa', not {state_layout!r}")
        self.state_layout = state_layout
        self.rng = rng
        self.seed = 1984  # Kernel.cu:175 seed base; the Philox key in perf mode
        self.frame = 0    # Philox frame counter (the XORWOW streams carry over in `state` instead)
        if not torch.cuda.is_available():
            raise RTError("no HIP device visible: librt_hip.so renders on MI355X only")
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        torch.cuda.set_device(self.device)
        check(lib().rt_set_device(self.device.index or 0), "rt_set_device")
        self.width, self.height = width, height
        self.band_rows = band_rows or height
        self.num_ranks, self.rank = num_ranks, rank
        self.rows = band_rows_of(height, self.band_rows, num_ranks, rank)
        self.local_rows = len(self.rows)
        n = width * self.local_rows
        # InitCudaBuffers (CudaLayer.cpp:68-74): RGBA8 framebuffer + one 48-byte curandState per pixel
        # (none in Philox mode)
        self.pos = torch.zeros(n, dtype=torch.int32, device=self.device)
        words = n * abi.STATE_WORDS if state_layout == "curand" else 6 * int(lib().rt_soa_plane_words(width, self.local_rows))
        self.state = torch.zeros(words, dtype=torch.int32, device=self.device) if rng == "xorwow" else None
        self.counters = torch.zeros(abi.COUNTERS_WORDS, dtype=torch.int64, device=self.device)
        self.radiance = None
        self.accum = None
        self._accum_restart = False  # the next accumulating frame restarts the sums (RT_FLAG_ACCUMULATE_RESET)

    def tiling(self) -> abi.Tiling:
        return abi.Tiling(self.band_rows, self.num_ranks, self.rank, self.local_rows)

    def stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def render_init(self, seed_base: int = 1984) -> None:
        """RenderInit: curand_init(seed_base + global pixel index, 0, 0) (Kernel.cu:166-176); in Philox mode
        the seed becomes the Philox key and the frame counter restarts."""
        self.seed, self.frame = seed_base, 0
        if self.state is None:
            return
        t = self.tiling()
        init = lib().rt_render_init_soa if self.state_layout == "soa" else lib().rt_render_init
        check(init(C.c_void_p(self.state.data_ptr()), self.width, self.height, C.byref(t), seed_base,
                   C.c_void_p(self.stream())), "rt_render_init")

    def render(self, scene: DeviceScene, spp: int, max_depth: int, inputs: abi.InputStruct, flags: int = 0,
               radiance: bool = False, count: bool = True, frame: int | None = None) -> torch.Tensor:
        """One frame (Kernel.cu:102-158), asynchronous on torch's current stream; returns `pos`.  Philox
        mode draws frame `frame` (default: the next frame counter value) of every pixel's stream."""
        if radiance and self.radiance is None:
            self.radiance = torch.zeros(self.width * self.local_rows * 4, dtype=torch.float32, device=self.device)
        if flags & abi.RT_FLAG_ACCUMULATE:
            if self.accum is None:
                # zeroed once: the first frame (RT_FLAG_ACCUMULATE_RESET) writes every pixel it renders, but with
                # RT_FLAG_FAITHFUL_GRID the pixels outside whole 16×16 blocks are never rendered and must read 0
                self.accum = torch.zeros(self.width * self.local_rows * 4, dtype=torch.float32, device=self.device)
                self._accum_restart = True
            if self._accum_restart:
                flags |= abi.RT_FLAG_ACCUMULATE_RESET
                self._accum_restart = False
        a = abi.RenderArgs()
        a.pos = self.pos.data_ptr()
        a.radiance = self.radiance.data_ptr() if radiance else None
        a.accum = self.accum.data_ptr() if self.accum is not None and flags & abi.RT_FLAG_ACCUMULATE else None
        a.state = self.state.data_ptr() if self.state is not None else None
        a.counters = self.counters.data_ptr() if count else None
        a.width, a.height = self.width, self.height
        a.samples_per_pixel, a.max_depth = spp, max_depth
        if self.rng == "philox":
            flags |= abi.RT_FLAG_RNG_PHILOX
            if frame is None:
                frame = self.frame
                if not flags & abi.RT_FLAG_NO_STATE_WRITEBACK:
                    self.frame += 1  # the next frame draws fresh numbers, as the XORWOW streams advance
            a.rng_seed, a.rng_frame = self.seed, frame
        if self.state_layout == "soa" and self.state is not None:
            flags |= abi.RT_FLAG_STATE_SOA
        a.flags = flags
        a.tiling = self.tiling()
        a.inputs = inputs
        check(lib().rt_render(scene.handle, C.byref(a), C.c_void_p(self.stream())), "rt_render")
        return self.pos

    def reset_accumulation(self) -> None:
        """Restart the progressive sums (camera move, scene edit): the next accumulating frame passes
        RT_FLAG_ACCUMULATE_RESET, which writes the accumulator without reading it — no fill kernel."""
        self._accum_restart = True

    def image(self) -> np.ndarray:
        """Local framebuffer as (local_rows, W) uint32 RGBA8 (row 0 = bottom of the image)."""
        return self.pos.cpu().numpy().view(np.uint32).reshape(self.local_rows, self.width)

    def states(self) -> np.ndarray:
        """The XORWOW states as (pixels, 12) rt_curand_state words (the SoA planes transposed into words 0-5;
        words 6-11, the Box-Muller fields the path never uses, zero)."""
        w = self.state.cpu().numpy().view(np.uint32)
        if self.state_layout == "curand":
            return w.reshape(-1, abi.STATE_WORDS)
        ly, x = np.divmod(np.arange(self.width * self.local_rows), self.width)
        idx = ((ly >> 3) * ((self.width + 7) >> 3) + (x >> 3)) * 64 + (ly & 7) * 8 + (x & 7)  # soa_index
        out = np.zeros((idx.size, abi.STATE_WORDS), dtype=np.uint32)
        out[:, :6] = w.reshape(6, -1)[:, idx].T
        return out

    def radiance_image(self) -> np.ndarray:
        return self.radiance.cpu().numpy().reshape(self.local_rows, self.width, 4)


class TiledRenderer:
    """Single-process multi-device tiling through librt_hip.so (rt_tiled_*): rank r renders the block-cyclic
    row bands b ≡ r (mod N) on devices[r] and copies them into their rows of the gathered frame (one strided
    peer copy per rank).  The C-ABI path a C++ viewer uses for the north star's 8-GPU split, without torch."""

    def __init__(self, width: int, height: int, devices, scene: Scene, band_rows: int = 16, rng: str = "xorwow",
                 seed: int = 1984):
        if not torch.cuda.is_available():
            raise RTError("no HIP device visible: librt_hip.so renders on MI355X only")
        self.width, self.height = width, height
        self.devices = list(devices)
        self._devs = (C.c_int * len(self.devices))(*self.devices)
        d = abi.TiledDesc(C.cast(self._devs, C.POINTER(C.c_int)), len(self.devices), band_rows, width, height,
                          abi.RT_FLAG_RNG_PHILOX if rng == "philox" else 0, 0, seed)
        self._scene_desc = scene.desc()
        self.handle = C.c_void_p()
        check(lib().rt_tiled_create(C.byref(d), C.byref(self._scene_desc), C.byref(self.handle)), "rt_tiled_create")
        self.pos = torch.zeros(width * height, dtype=torch.int32, device=torch.device("cuda", self.devices[0]))
        self.timing = abi.TiledTiming()

    def render(self, spp: int, max_depth: int, inputs: abi.InputStruct, flags: int = 0, frame: int | None = None,
               pos: torch.Tensor | None = None) -> torch.Tensor:
        """One frame over all ranks, gathered into `pos` (default: a buffer on devices[0]); synchronous."""
        out = self.pos if pos is None else pos
        f = abi.TiledFrame(out.data_ptr(), spp, max_depth, flags, frame or 0, 0 if frame is None else 1, 0, inputs)
        check(lib().rt_tiled_render(self.handle, C.byref(f), C.byref(self.timing)), "rt_tiled_render")
        return out

    def image(self) -> np.ndarray:
        return self.pos.cpu().numpy().view(np.uint32).reshape(self.height, self.width)

    def close(self) -> None:
        if self.handle:
            lib().rt_tiled_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
