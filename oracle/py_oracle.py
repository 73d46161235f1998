"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU restatement (oracle/build/liboracle.so).

Used by tests/ (as the checker), __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product
never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from cudaraytracer_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

_lib = None


class Counters(C.Structure):
    _fields_ = [("rays", C.c_ulonglong), ("box_tests", C.c_ulonglong), ("prim_tests", C.c_ulonglong),
                ("primary", C.c_ulonglong), ("rect_tests", C.c_ulonglong)]


class Hit(C.Structure):
    _fields_ = [("hit", C.c_int), ("t", C.c_float), ("p", C.c_float * 3), ("normal", C.c_float * 3),
                ("u", C.c_float), ("v", C.c_float), ("front_face", C.c_int)]


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_native = {}


def native_lib(out_dir: str) -> C.CDLL:
    """The -O3 -march=native build of the same source (CPU baseline, `make -C oracle native`), built into
    out_dir on the host that runs it."""
    if out_dir not in _native:
        subprocess.run(["make", "-s", "-C", HERE, "native", f"NATIVE_OUT={out_dir}"], check=True)
        _native[out_dir] = _declare(C.CDLL(os.path.join(out_dir, "liboracle.so")))
    return _native[out_dir]


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = _declare(C.CDLL(LIB_PATH))
    return _lib


def _declare(L: C.CDLL) -> C.CDLL:
    if True:
        vp = C.c_void_p
        L.orc_curand_init.argtypes = [C.c_ulonglong, vp]
        L.orc_xorwow_seed.argtypes = [C.c_ulonglong, C.c_uint, C.c_uint, C.c_uint, C.c_uint, vp]
        L.orc_curand.argtypes = [vp]
        L.orc_curand.restype = C.c_uint
        L.orc_curand_uniform.argtypes = [vp]
        L.orc_curand_uniform.restype = C.c_float
        L.orc_scene_build.argtypes = [C.POINTER(abi.SceneDesc)]
        L.orc_scene_build.restype = vp
        L.orc_scene_free.argtypes = [vp]
        L.orc_scene_num_nodes.argtypes = [vp]
        L.orc_scene_depth.argtypes = [vp]
        L.orc_scene_set_exact.argtypes = [vp, C.c_int]
        L.orc_render_init.argtypes = [vp, C.c_uint, C.c_uint, C.c_ulonglong, C.c_int]
        L.orc_render.argtypes = [vp, vp, vp, vp, C.c_uint, C.c_uint, C.c_uint, C.c_uint, vp, C.POINTER(abi.InputStruct),
                                 C.c_int, C.c_uint, C.c_uint, C.c_uint, C.c_int, C.c_int, C.c_int, C.c_ulonglong,
                                 C.c_uint, C.POINTER(Counters)]
        L.orc_philox4x32_10.argtypes = [C.POINTER(C.c_uint), C.POINTER(C.c_uint), C.POINTER(C.c_uint)]
        L.orc_philox_uniform_at.argtypes = [C.c_ulonglong, C.c_uint, C.c_uint, C.c_uint]
        L.orc_philox_uniform_at.restype = C.c_float
        L.orc_hittable_hit.argtypes = [C.POINTER(abi.HittableDesc), C.POINTER(C.c_float), C.POINTER(C.c_float),
                                       C.c_float, C.c_float, C.POINTER(Hit)]
        L.orc_scatter.argtypes = [C.POINTER(abi.MaterialDesc), C.POINTER(C.c_float), C.POINTER(C.c_float),
                                  C.POINTER(Hit), vp, C.POINTER(C.c_float), C.POINTER(C.c_float),
                                  C.POINTER(C.c_float), C.POINTER(C.c_int), C.c_int]
        L.orc_rgb_to_int.argtypes = [C.c_float, C.c_float, C.c_float]
        L.orc_rgb_to_int.restype = C.c_uint
    return L


class OracleScene:
    """exact=False: the reference BVH and its AABB culling (Hittable.cuh:303-439); exact=True: geometric
    closest hit over all active primitives (see orc_scene_set_exact)."""

    def __init__(self, scene, exact: bool = False, library: C.CDLL | None = None):
        self.scene = scene
        self._lib = library or lib()
        self._desc = scene.desc()
        self.handle = self._lib.orc_scene_build(C.byref(self._desc))
        self._lib.orc_scene_set_exact(self.handle, 1 if exact else 0)

    @property
    def depth(self) -> int:
        return lib().orc_scene_depth(self.handle)

    def __del__(self):
        try:
            self._lib.orc_scene_free(self.handle)
        except Exception:
            pass


def init_states(width: int, height: int, seed_base: int = 1984, full: bool = True) -> np.ndarray:
    st = np.zeros((width * height, abi.STATE_WORDS), dtype=np.uint32)
    lib().orc_render_init(st.ctypes.data, width, height, seed_base, 1 if full else 0)
    return st


def render(oscene: OracleScene, width: int, height: int, spp: int, depth: int, inputs: abi.InputStruct,
           states: np.ndarray, faithful_grid: bool = False, rows: tuple | None = None, threads: int = 0,
           rius_order: int = 1, radiance: bool = False, row_step: int = 1, philox: bool = False,
           seed: int = 1984, frame: int = 0, accum: np.ndarray | None = None, library: C.CDLL | None = None):
    """One frame; returns (pos (H, W) uint32, radiance (H, W, 4) or None, Counters).  `states` advances
    (XORWOW mode); with philox=True the pixels draw from their (seed, pixel, frame) Philox streams and
    `states` may be None.  `accum` (H·W·4 float32, updated in place): progressive accumulation
    (RT_FLAG_ACCUMULATE semantics)."""
    if accum is not None:
        assert accum.dtype == np.float32 and accum.size == width * height * 4 and accum.flags.c_contiguous
    pos = np.zeros(width * height, dtype=np.uint32)
    rad = np.zeros(width * height * 4, dtype=np.float32) if radiance else None
    cnt = Counters()
    r0, r1 = rows if rows else (0, height)
    (library or lib()).orc_render(oscene.handle, pos.ctypes.data, rad.ctypes.data if rad is not None else None,
                     accum.ctypes.data if accum is not None else None, width, height,
                     spp, depth, states.ctypes.data if states is not None else None, C.byref(inputs),
                     1 if faithful_grid else 0, r0, r1, row_step, threads, rius_order, 1 if philox else 0, seed, frame,
                     C.byref(cnt))
    return pos.reshape(height, width), (rad.reshape(height, width, 4) if rad is not None else None), cnt
