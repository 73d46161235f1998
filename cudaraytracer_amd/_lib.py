"""Loader for the in-tree librt_hip.so (built by `__graft_entry__.build()` / `make -C cudaraytracer_amd/csrc`).

There is no fallback: if the library is missing or fails to load, importing the renderer raises.
"""
from __future__ import annotations

import ctypes as C
import os

from . import abi

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "librt_hip.so")
# A/B experiments only: RT_HIP_LIB names another in-tree build of the same library (tools/ab_builds.sh).
LIB_PATH = os.environ.get("RT_HIP_LIB", LIB_PATH)

# Every symbol include/rt_hip.h declares (checked by tests/test_abi.py).
EXPORTED = [
    "LaunchKernel",
    "LaunchRandInit",
    "LaunchRenderInit",
    "rt_last_error",
    "rt_version",
    "rt_abi_version",
    "rt_set_launch_flags",
    "rt_set_device",
    "rt_scene_create",
    "rt_scene_from_reference_graph",
    "rt_scene_update_materials",
    "rt_scene_destroy",
    "rt_scene_get_info",
    "rt_render_init",
    "rt_render_init_soa",
    "rt_soa_plane_words",
    "rt_render",
    "rt_tiled_create",
    "rt_tiled_render",
    "rt_tiled_destroy",
    "rt_gl_register_texture",
    "rt_gl_copy_image",
    "rt_gl_unregister",
    "rt_copy_image_to_host",
    "rt_write_ppm",
    "rt_set_timing",
    "rt_set_wave_trace",
    "rt_set_tile_order",
    "rt_set_pixel_cost",
    "rt_set_ray_dump",
    "rt_trace_rays",
    "rt_last_kernel_ms",
    "rt_last_variant",
    "rt_last_launch_host_ms",
    "rt_set_variant",
    "rt_set_tuning",
    "rt_glibc_srand",
    "rt_glibc_rand_next",
    "rt_builtin_scene",
    "rt_camera_inputs",
    "rt_procedural_texture",
    "rt_reference_graph_flatten",
    "rt_build_host_tables",
]

_lib = None


class RTError(RuntimeError):
    pass


def _declare(lib: C.CDLL) -> None:
    P = C.POINTER
    vp = C.c_void_p
    lib.rt_last_error.restype = C.c_char_p
    lib.rt_version.restype = C.c_char_p
    lib.rt_set_launch_flags.argtypes = [C.c_uint32]
    lib.rt_set_device.argtypes = [C.c_int]
    lib.rt_scene_create.argtypes = [P(abi.SceneDesc), P(vp)]
    lib.rt_scene_from_reference_graph.argtypes = [vp, P(vp)]
    lib.rt_scene_update_materials.argtypes = [vp, P(abi.MaterialDesc), C.c_uint32]
    lib.rt_scene_destroy.argtypes = [vp]
    lib.rt_scene_get_info.argtypes = [vp, P(abi.SceneInfo)]
    lib.rt_render_init.argtypes = [vp, C.c_uint32, C.c_uint32, P(abi.Tiling), C.c_uint64, vp]
    lib.rt_render_init_soa.argtypes = [vp, C.c_uint32, C.c_uint32, P(abi.Tiling), C.c_uint64, vp]
    lib.rt_soa_plane_words.argtypes = [C.c_uint32, C.c_uint32]
    lib.rt_soa_plane_words.restype = C.c_uint64
    lib.rt_render.argtypes = [vp, P(abi.RenderArgs), vp]
    lib.rt_set_timing.argtypes = [C.c_int]
    lib.rt_tiled_create.argtypes = [P(abi.TiledDesc), P(abi.SceneDesc), P(vp)]
    lib.rt_tiled_render.argtypes = [vp, P(abi.TiledFrame), P(abi.TiledTiming)]
    lib.rt_tiled_destroy.argtypes = [vp]
    lib.rt_gl_register_texture.argtypes = [C.c_uint32, C.c_uint32, P(vp)]
    lib.rt_gl_copy_image.argtypes = [vp, vp, C.c_uint32, C.c_uint32, vp]
    lib.rt_gl_unregister.argtypes = [vp]
    lib.rt_copy_image_to_host.argtypes = [vp, vp, C.c_uint32, C.c_uint32, C.c_int, vp]
    lib.rt_write_ppm.argtypes = [C.c_char_p, vp, C.c_uint32, C.c_uint32, C.c_int]
    lib.rt_set_wave_trace.argtypes = [C.c_void_p, C.c_uint64]
    lib.rt_set_tile_order.argtypes = [C.c_void_p]
    lib.rt_set_pixel_cost.argtypes = [C.c_void_p, C.c_uint64]
    lib.rt_set_ray_dump.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]
    lib.rt_trace_rays.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    lib.rt_last_kernel_ms.restype = C.c_float
    lib.rt_last_variant.restype = C.c_int
    lib.rt_last_launch_host_ms.restype = C.c_float
    lib.rt_set_variant.argtypes = [C.c_int]
    lib.rt_set_tuning.argtypes = [C.c_int, C.c_int]
    lib.rt_glibc_srand.argtypes = [P(abi.GlibcRand), C.c_uint32]
    lib.rt_glibc_rand_next.argtypes = [P(abi.GlibcRand)]
    lib.rt_glibc_rand_next.restype = C.c_int32
    lib.rt_builtin_scene.argtypes = [C.c_int, C.c_uint32, P(abi.HittableDesc), P(C.c_uint32),
                                     P(abi.MaterialDesc), P(C.c_uint32)]
    lib.rt_procedural_texture.argtypes = [C.c_int, C.c_int32, C.c_int32, C.c_void_p]
    F3P = P(C.c_float)
    lib.rt_camera_inputs.argtypes = [F3P, F3P, F3P, C.c_float, C.c_float, C.c_float, F3P, F3P, P(abi.InputStruct)]
    lib.rt_reference_graph_flatten.argtypes = [vp, P(abi.HittableDesc), P(C.c_uint32), P(abi.MaterialDesc),
                                               P(C.c_uint32), P(abi.ImageDesc), P(C.c_uint32)]
    lib.rt_build_host_tables.argtypes = [P(abi.SceneDesc), P(C.c_float), P(C.c_float), P(C.c_float),
                                         P(C.c_int32), P(abi.HostTablesInfo)]
    lib.LaunchKernel.argtypes = [vp, C.c_uint, C.c_uint, C.c_uint, C.c_uint, vp, vp, abi.InputStruct]
    lib.LaunchKernel.restype = None
    lib.LaunchRandInit.argtypes = [vp]
    lib.LaunchRandInit.restype = None
    lib.LaunchRenderInit.argtypes = [abi.Dim3, abi.Dim3, C.c_uint, C.c_uint, vp]
    lib.LaunchRenderInit.restype = None


def lib() -> C.CDLL:
    """The loaded librt_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RTError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        handle = C.CDLL(LIB_PATH)
        _declare(handle)
        _lib = handle
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().rt_last_error().decode(errors="replace")
        raise RTError(f"{what} failed: {abi.STATUS.get(rc, rc)}: {msg}")
