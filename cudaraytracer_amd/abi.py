"""ctypes mirror of include/rt_hip.h (the C ABI of librt_hip.so).

Plain data types only: these structures are the drop-in boundary's argument types, shared by the
product wrapper (`cudaraytracer_amd.renderer`) and by the tests that feed the same inputs to the oracle.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

# enums (Hittable.cuh:30-38, Material.cuh:6-12, Texture.cuh:6-10)
RT_SPHERE, RT_XYRECT, RT_XZRECT, RT_YZRECT = 0, 1, 2, 3
RT_LAMBERTIAN, RT_METAL, RT_DIELECTRIC, RT_DIFFUSELIGHT = 0, 1, 2, 3
RT_CONSTANT, RT_CHECKER, RT_IMAGE = 0, 1, 2

RT_FLAG_FAITHFUL_GRID = 1 << 0
RT_FLAG_NO_STATE_WRITEBACK = 1 << 1
RT_FLAG_ACCUMULATE = 1 << 2
RT_FLAG_RIUS_LEFT_TO_RIGHT = 1 << 3
RT_FLAG_COUNT_TESTS = 1 << 4
RT_FLAG_RNG_PHILOX = 1 << 5
RT_FLAG_STATE_SOA = 1 << 6
RT_FLAG_ACCUMULATE_RESET = 1 << 7
COUNTERS_WORDS = 24  # RT_COUNTERS_WORDS: the counters buffer with RT_FLAG_COUNT_TESTS
PHILOX_MAX_SPP = 16384  # RT_PHILOX_MAX_SPP
# rt_set_tuning keys (rt_tuning_key in include/rt_hip.h)
RT_TUNE_REGEN_THRESHOLD, RT_TUNE_LEAF_MAX, RT_TUNE_PERSISTENT_WAVES, RT_TUNE_SAH_TRAVERSAL = 0, 1, 2, 3
RT_TUNE_LDS_PAD, RT_TUNE_ADAPTIVE_ORDER, RT_TUNE_TEXEL_LAYOUT, RT_TUNE_QUEUE_CHUNK = 4, 5, 6, 7
RT_TUNE_QUEUE_STRIDE, RT_TUNE_REGEN_LIVE_FRAC, RT_TUNE_LEAF_BREAK, RT_TUNE_RIUS_TRIPS = 8, 9, 10, 11
RT_TUNE_FLAT_MAX = 12
RT_TUNE_QUEUE_PREFETCH = 13
RT_TUNE_QUEUE_GUIDE = 14
RT_TUNE_QUEUE_MIN_CHUNK = 15
RT_TUNE_RIUS_TRIPS_PERSISTENT = 16
RT_TUNE_PREFETCH_STOP = 17
RT_TUNE_PERSISTENT_GROUP = 18  # persistent flat kernel: 16-wave workgroups with static tile shares (1) or not (0)
RT_TUNE_GROUP_ORDER = 20  # ... the shares' tiles interleaved (0) or in golden-ratio order (1)
RT_TUNE_QUEUE_RESET = 21  # 1 = rt_render memsets the persistent queue slot per launch
RT_TUNE_GROUP_CHUNK = 22  # ... positions per chunk of the workgroup chunk queue (group mode 2)
RT_TUNE_GROUP_LINGER_US = 23  # ... a finished workgroup waits this long (us) for the grid's others before exiting
RT_TUNE_GROUP_WAVES = 24  # ... waves per workgroup of the persistent flat kernel's group builds (4/8/12/16)
RT_TUNE_GROUP_TAIL = 19  # ... permille of the tiles left to the per-wave queue behind the shares

STATUS = {
    0: "RT_OK",
    -1: "RT_ERR_INVALID_ARGUMENT",
    -2: "RT_ERR_INVALID_SCENE",
    -3: "RT_ERR_OUT_OF_MEMORY",
    -4: "RT_ERR_DEVICE",
    -5: "RT_ERR_LAUNCH",
    -6: "RT_ERR_UNSUPPORTED",
}

F3 = C.c_float * 3


class TextureDesc(C.Structure):
    _fields_ = [("type", C.c_int32), ("image", C.c_int32), ("color", F3), ("color2", F3)]


class MaterialDesc(C.Structure):
    _fields_ = [
        ("type", C.c_int32),
        ("fuzz", C.c_float),
        ("ir", C.c_float),
        ("light_intensity", C.c_int32),
        ("albedo", TextureDesc),
    ]


class HittableDesc(C.Structure):
    _fields_ = [
        ("type", C.c_int32),
        ("is_active", C.c_int32),
        ("center", F3),
        ("radius", C.c_float),
        ("width", C.c_float),
        ("height", C.c_float),
        ("material", C.c_int32),
        ("reserved", C.c_int32),
    ]


class ImageDesc(C.Structure):
    _fields_ = [("data", C.c_void_p), ("width", C.c_int32), ("height", C.c_int32)]


class SceneDesc(C.Structure):
    _fields_ = [
        ("hittables", C.POINTER(HittableDesc)),
        ("num_hittables", C.c_uint32),
        ("materials", C.POINTER(MaterialDesc)),
        ("num_materials", C.c_uint32),
        ("images", C.POINTER(ImageDesc)),
        ("num_images", C.c_uint32),
    ]


class InputStruct(C.Structure):
    """InputStruct (Utils/SharedStructs.h:3-24), 72 bytes."""

    _fields_ = [
        ("origin", F3),
        ("orientation", F3),
        ("up", F3),
        ("far_plane", C.c_float),
        ("near_plane", C.c_float),
        ("fov", C.c_float),
        ("background_start", F3),
        ("background_end", F3),
    ]


class CurandState(C.Structure):
    """curandStateXORWOW layout, 48 bytes."""

    _fields_ = [
        ("d", C.c_uint32),
        ("v", C.c_uint32 * 5),
        ("boxmuller_flag", C.c_int32),
        ("boxmuller_flag_double", C.c_int32),
        ("boxmuller_extra", C.c_float),
        ("pad_", C.c_uint32),
        ("boxmuller_extra_double", C.c_double),
    ]


class Dim3(C.Structure):
    _fields_ = [("x", C.c_uint32), ("y", C.c_uint32), ("z", C.c_uint32)]


class Tiling(C.Structure):
    _fields_ = [
        ("band_rows", C.c_uint32),
        ("num_ranks", C.c_uint32),
        ("rank", C.c_uint32),
        ("local_rows", C.c_uint32),
    ]


class RenderArgs(C.Structure):
    _fields_ = [
        ("pos", C.c_void_p),
        ("radiance", C.c_void_p),
        ("accum", C.c_void_p),
        ("state", C.c_void_p),
        ("counters", C.c_void_p),
        ("width", C.c_uint32),
        ("height", C.c_uint32),
        ("samples_per_pixel", C.c_uint32),
        ("max_depth", C.c_uint32),
        ("flags", C.c_uint32),
        ("reserved", C.c_uint32),
        ("tiling", Tiling),
        ("inputs", InputStruct),
        ("rng_seed", C.c_uint64),
        ("rng_frame", C.c_uint32),
        ("reserved2", C.c_uint32),
    ]


class TiledDesc(C.Structure):
    _fields_ = [("devices", C.POINTER(C.c_int)), ("num_ranks", C.c_uint32), ("band_rows", C.c_uint32),
                ("width", C.c_uint32), ("height", C.c_uint32), ("flags", C.c_uint32), ("reserved", C.c_uint32),
                ("seed", C.c_uint64)]


class TiledFrame(C.Structure):
    _fields_ = [("pos", C.c_void_p), ("samples_per_pixel", C.c_uint32), ("max_depth", C.c_uint32),
                ("flags", C.c_uint32), ("rng_frame", C.c_uint32), ("rng_frame_set", C.c_uint32),
                ("reserved", C.c_uint32), ("inputs", InputStruct)]


class TiledTiming(C.Structure):
    _fields_ = [("render_ms", C.c_float), ("gather_ms", C.c_float), ("total_ms", C.c_float), ("reserved", C.c_uint32),
                ("rays", C.c_uint64)]


class SceneInfo(C.Structure):
    _fields_ = [
        ("num_primitives", C.c_uint32),
        ("num_nodes", C.c_uint32),
        ("num_materials", C.c_uint32),
        ("bvh_depth", C.c_uint32),
        ("device_bytes", C.c_uint64),
    ]


class HostTablesInfo(C.Structure):
    _fields_ = [("num_nodes", C.c_uint32), ("num_prims", C.c_uint32), ("num_materials", C.c_uint32),
                ("depth", C.c_uint32)]


class GlibcRand(C.Structure):
    _fields_ = [("r", C.c_int32 * 34), ("idx", C.c_uint32)]


# numpy views of the RNG-state layout: 12 uint32 words per state (d, v0..v4, flags, extra, pad, double)
STATE_WORDS = 12
assert C.sizeof(CurandState) == 48
assert C.sizeof(InputStruct) == 72
assert C.sizeof(HittableDesc) == 40
assert C.sizeof(MaterialDesc) == 48
assert C.sizeof(TextureDesc) == 32


def make_inputs(origin, orientation, up, far_plane, near_plane, fov, bg_start, bg_end) -> InputStruct:
    s = InputStruct()
    s.origin[:] = [float(v) for v in origin]
    s.orientation[:] = [float(v) for v in orientation]
    s.up[:] = [float(v) for v in up]
    s.far_plane = far_plane
    s.near_plane = near_plane
    s.fov = fov
    s.background_start[:] = [float(v) for v in bg_start]
    s.background_end[:] = [float(v) for v in bg_end]
    return s


def states_as_words(states: np.ndarray) -> np.ndarray:
    """View an (N,) buffer of 48-byte states as (N, 12) uint32."""
    return states.view(np.uint32).reshape(-1, STATE_WORDS)
