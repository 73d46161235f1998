"""CPU tests of the C-ABI boundary: librt_hip.so loads, exports every function include/*.h declares, and the
struct layouts match the reference's (InputStruct 72 B, curandState 48 B, graph node sizes)."""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

from cudaraytracer_amd import abi
from cudaraytracer_amd._lib import EXPORTED, LIB_PATH, lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions() -> set:
    names = set()
    for fn in os.listdir(os.path.join(ROOT, "include")):
        if not fn.endswith(".h"):
            continue
        text = open(os.path.join(ROOT, "include", fn)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\(", text, flags=re.M):
            name = m.group(1)
            if name not in {"if", "sizeof", "static_assert", "typedef"}:
                names.add(name)
    return names


def test_library_loads():
    assert os.path.exists(LIB_PATH)
    assert lib().rt_version().startswith(b"librt_hip")


def test_abi_version_matches_the_header():
    """RT_COUNTERS_WORDS grew with RT_FLAG_COUNT_TESTS; the ABI version names such changes, and the library
    reports the version of the header it was built from."""
    hdr = open(os.path.join(ROOT, "include", "rt_hip.h")).read()
    m = re.search(r"#define RT_ABI_VERSION (\d+)", hdr)
    assert m and lib().rt_abi_version() == int(m.group(1)) >= 6
    assert re.search(r"#define RT_COUNTERS_WORDS (\d+)u", hdr).group(1) == str(abi.COUNTERS_WORDS)


def test_launch_flags_accept_only_the_fill_order():
    """rt_set_launch_flags (LaunchKernel's Random() fill order): RT_FLAG_RIUS_LEFT_TO_RIGHT is
    accepted and returned as the previous value; any other bit is refused without changing the setting."""
    L = lib()
    prev = L.rt_set_launch_flags(abi.RT_FLAG_RIUS_LEFT_TO_RIGHT)
    try:
        assert prev in (0, abi.RT_FLAG_RIUS_LEFT_TO_RIGHT)
        assert L.rt_set_launch_flags(abi.RT_FLAG_RIUS_LEFT_TO_RIGHT | abi.RT_FLAG_RNG_PHILOX) < 0
        assert L.rt_set_launch_flags(0) == abi.RT_FLAG_RIUS_LEFT_TO_RIGHT
    finally:
        L.rt_set_launch_flags(prev)


def test_every_declared_symbol_is_exported():
    decl = declared_functions()
    assert decl == set(EXPORTED), (decl ^ set(EXPORTED))
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = decl - exported
    assert not missing, missing
    for name in decl:
        assert hasattr(lib(), name)


def test_struct_layouts():
    assert C.sizeof(abi.InputStruct) == 72  # SharedStructs.h:3-24
    assert C.sizeof(abi.CurandState) == 48  # curandStateXORWOW
    assert C.sizeof(abi.Dim3) == 12
    assert C.sizeof(abi.HittableDesc) == 40 and C.sizeof(abi.MaterialDesc) == 48


def test_error_reporting_without_device():
    h = C.c_void_p()
    assert lib().rt_scene_create(None, C.byref(h)) == -1
    assert b"NULL" in lib().rt_last_error()
    assert lib().rt_render(None, None, None) == -1


def test_soa_plane_words_cover_whole_tiles():
    """RT_FLAG_STATE_SOA planes hold whole 8x8 tiles (include/rt_hip.h rt_soa_plane_words)."""
    from cudaraytracer_amd._lib import lib
    assert lib().rt_soa_plane_words(1920, 1080) == 1920 * 1080
    assert lib().rt_soa_plane_words(100, 37) == 13 * 5 * 64
    assert lib().rt_soa_plane_words(7680, 544) == 960 * 68 * 64
    assert lib().rt_soa_plane_words(1, 1) == 64
    assert lib().rt_soa_plane_words(0, 5) == 0


def test_philox_spp_limit_is_rejected_before_any_device_work():
    """RT_FLAG_RNG_PHILOX reads sample s's window at word s << 18 of the pixel's stream (include/rt_hip.h
    RT_PHILOX_MAX_SPP): above 2^14 samples the oracle's 32-bit word counter would wrap, so rt_render rejects the
    call — checked here before the scene is touched, so no GPU is needed."""
    a = abi.RenderArgs()
    a.width, a.height, a.max_depth = 8, 8, 4
    a.tiling.band_rows, a.tiling.num_ranks, a.tiling.rank, a.tiling.local_rows = 8, 1, 0, 8
    a.flags = abi.RT_FLAG_RNG_PHILOX
    dummy = C.create_string_buffer(64)  # never dereferenced: the limit is checked first
    for spp in (16385, 1 << 16, 1 << 20):
        a.samples_per_pixel = spp
        assert lib().rt_render(C.cast(dummy, C.c_void_p), C.byref(a), None) == -1, spp
        assert b"RT_PHILOX_MAX_SPP" in lib().rt_last_error()
