"""Headless output and the display step after the kernel (CudaLayer.cpp:89-90, 379-386, 402).

CPU: rt_write_ppm against the bytes numpy derives from a golden frame (upright: buffer row 0 is the bottom of
the image) and argument checks of the GL interop entry points (which need a GL context to do anything).
GPU: the host-staging fallback (rt_copy_image_to_host) returns the rendered frame, flipped upright on request.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from cudaraytracer_amd._lib import lib
from helpers import load_golden


def _ppm_bytes(img: np.ndarray, flip: bool) -> bytes:
    h, w = img.shape
    rows = img[::-1] if flip else img
    rgb = np.ascontiguousarray(rows).view(np.uint8).reshape(h, w, 4)[..., :3]
    return f"P6\n{w} {h}\n255\n".encode() + rgb.tobytes()


@pytest.mark.parametrize("flip", [0, 1])
def test_write_ppm_matches_golden_frame(tmp_path, flip):
    img = np.ascontiguousarray(load_golden("c2_rtiow_192x112_s16")["pos"].astype(np.uint32))
    path = tmp_path / "frame.ppm"
    h, w = img.shape
    assert lib().rt_write_ppm(str(path).encode(), img.ctypes.data, w, h, flip) == 0
    assert path.read_bytes() == _ppm_bytes(img, bool(flip))
    if flip:  # the sky (bright blue-white) is at the top of the upright image: row H-1 of the buffer
        data = path.read_bytes()[len(f"P6\n{w} {h}\n255\n"):]
        top = np.frombuffer(data[: 3 * w], np.uint8).reshape(w, 3)
        bottom = np.frombuffer(data[-3 * w:], np.uint8).reshape(w, 3)
        assert top[:, 2].mean() > bottom[:, 2].mean()


def test_display_entry_points_reject_bad_arguments(tmp_path):
    out = C.c_void_p()
    assert lib().rt_gl_register_texture(0, 0x0DE1, C.byref(out)) == -1  # texture name 0
    assert lib().rt_gl_register_texture(5, 0x0DE1, None) == -1
    assert lib().rt_gl_copy_image(None, None, 4, 4, None) == -1
    assert lib().rt_gl_unregister(None) == 0
    assert lib().rt_copy_image_to_host(None, None, 4, 4, 0, None) == -1
    assert lib().rt_write_ppm(str(tmp_path / "x.ppm").encode(), None, 4, 4, 0) == -1
    assert lib().rt_write_ppm(b"/nonexistent-dir/x.ppm", (C.c_uint32 * 16)(), 4, 4, 0) == -1


@pytest.mark.gpu
@pytest.mark.parametrize("flip", [0, 1])
def test_host_staging_fallback_returns_the_frame(flip):
    import torch

    from cases import CASE_BY_NAME
    from cudaraytracer_amd import scenes
    from cudaraytracer_amd.renderer import DeviceScene, Renderer
    case = CASE_BY_NAME["c2_rtiow_ragged_100x37_s4"]
    cfg = case.cfg()
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    r.render(DeviceScene(scenes.builtin(cfg.scene)), cfg.spp, cfg.depth, cfg.inputs())
    torch.cuda.synchronize()
    host = np.zeros((cfg.height, cfg.width), np.uint32)
    assert lib().rt_copy_image_to_host(host.ctypes.data, C.c_void_p(r.pos.data_ptr()), cfg.width, cfg.height, flip,
                                       C.c_void_p(r.stream())) == 0
    want = load_golden(case.name)["pos"]
    np.testing.assert_array_equal(host, want[::-1] if flip else want)
