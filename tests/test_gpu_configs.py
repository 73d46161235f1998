"""BASELINE configurations 3, 4 and 5 exercised as configured (MI355X), against the oracle.

* C4 (7680×4320, 128 spp, depth 8, RTIOW, 8 ranks × 16-row bands): the shares of ranks 0, 3 and 7 render at
  full width on one GPU; strided full-width rows and their advanced cuRAND states equal the oracle's at the
  same GLOBAL pixel indices (Kernel.cu:119, 175).
* C5 (1920×1080, 1 spp, depth 4, textured spheres with three 8192×4096 RGB8 textures, progressive
  accumulation with the scripted moving camera and resets): every frame's RGBA8 image and float4
  accumulation buffer bit-exact against the oracle at a reduced size, and full-width row samples at full size.
* C3 (3840×2160, 256 spp, depth 16, Cornell box): row samples at the configured 256 spp.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd.renderer import DeviceScene, Renderer
from oracle import py_oracle as po

pytestmark = pytest.mark.gpu

THREADS = 16  # the GPU box's CPU share


def _global_rows(local_rows, band_rows, num_ranks, rank):
    return [((l // band_rows) * num_ranks + rank) * band_rows + l % band_rows for l in local_rows]


@pytest.fixture(scope="module")
def c4_oracle_states():
    cfg = scenes.CONFIGS["c4"]
    return po.init_states(cfg.width, cfg.height)  # 33 M × 48 B, seeded with the global pixel index


@pytest.mark.parametrize("rank", [0, 3, 7])
def test_c4_rank_share_rows_match_oracle(rank, c4_oracle_states):
    cfg = scenes.CONFIGS["c4"]
    assert (cfg.width, cfg.height, cfg.spp, cfg.depth) == (7680, 4320, 128, 8)
    sc = scenes.builtin(cfg.scene)
    r = Renderer(cfg.width, cfg.height, band_rows=16, num_ranks=8, rank=rank)
    assert r.local_rows == 540
    r.render_init()
    r.render(DeviceScene(sc), cfg.spp, cfg.depth, cfg.inputs())
    torch.cuda.synchronize()
    img = r.image()
    # local rows 16k + 7 for k = 0, 11, 22, 33: global rows (8k + rank)·16 + 7, evenly spaced → one oracle call
    local = [16 * k + 7 for k in (0, 11, 22, 33)]
    glob = _global_rows(local, 16, 8, rank)
    st = c4_oracle_states  # each rank's rows are disjoint: sharing the array across ranks is safe
    ref, _, _ = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st,
                          rows=(glob[0], cfg.height), row_step=glob[1] - glob[0], threads=THREADS)
    np.testing.assert_array_equal(img[local], ref[glob])
    states = r.states().reshape(r.local_rows, cfg.width, -1)
    np.testing.assert_array_equal(states[local, :, :6], st.reshape(cfg.height, cfg.width, -1)[glob, :, :6])
    assert np.all((img >> 24) == 0xFF)


def test_c4_rank_share_philox_rows_match_oracle():
    cfg = scenes.CONFIGS["c4"]
    sc = scenes.builtin(cfg.scene)
    r = Renderer(cfg.width, cfg.height, band_rows=16, num_ranks=8, rank=5, rng="philox")
    r.render_init()
    r.render(DeviceScene(sc), cfg.spp, cfg.depth, cfg.inputs(), frame=2)
    torch.cuda.synchronize()
    local = [16 * k + 9 for k in (2, 21)]
    glob = _global_rows(local, 16, 8, 5)
    ref, _, _ = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), None,
                          rows=(glob[0], cfg.height), row_step=glob[1] - glob[0], threads=THREADS, philox=True,
                          seed=1984, frame=2)
    np.testing.assert_array_equal(r.image()[local], ref[glob])


def _c5_schedule(frames: int):
    """Frame f looks from camera position f // 2 of the scripted orbit: two accumulated frames per camera
    position, then a reset (the viewer clears accumulation whenever the camera moves)."""
    out = []
    for f in range(frames):
        pos, fwd = scenes.moving_camera(f // 2, 60)
        out.append((scenes.camera_inputs(pos, fwd, scenes.CONFIGS["c5"].fov), f % 2 == 0))
    return out


@pytest.fixture(scope="module")
def c5_scene():
    cfg = scenes.CONFIGS["c5"]
    sc = cfg.scene_desc()  # three 8192×4096 RGB8 textures (≈100 MB each)
    assert [im.shape for im in sc.images] == [(4096, 8192, 3)] * 3
    return sc


@pytest.mark.parametrize("rng", ["xorwow", "philox"])
def test_c5_progressive_moving_camera_bit_exact(rng, c5_scene):
    cfg = scenes.CONFIGS["c5"].scaled(192, 108)
    assert (cfg.spp, cfg.depth) == (1, 4)
    ds = DeviceScene(c5_scene)
    r = Renderer(cfg.width, cfg.height, rng=rng)
    r.render_init()
    osc = po.OracleScene(c5_scene)
    st = po.init_states(cfg.width, cfg.height) if rng == "xorwow" else None
    acc = np.zeros(cfg.width * cfg.height * 4, np.float32)
    for frame, (inp, reset) in enumerate(_c5_schedule(8)):
        if reset:
            r.reset_accumulation()
            acc[:] = 0.0
        r.render(ds, cfg.spp, cfg.depth, inp, flags=abi.RT_FLAG_ACCUMULATE, frame=frame if rng == "philox" else None)
        torch.cuda.synchronize()
        ref, _, cnt = po.render(osc, cfg.width, cfg.height, cfg.spp, cfg.depth, inp, st, accum=acc,
                                philox=rng == "philox", frame=frame)
        np.testing.assert_array_equal(r.image(), ref, err_msg=f"frame {frame}")
        np.testing.assert_array_equal(r.accum.cpu().numpy(), acc, err_msg=f"frame {frame}")
    if st is not None:
        np.testing.assert_array_equal(r.states()[:, :6], st[:, :6])


def test_c5_full_size_progressive_rows_match_oracle(c5_scene):
    cfg = scenes.CONFIGS["c5"]
    ds = DeviceScene(c5_scene)
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    osc = po.OracleScene(c5_scene)
    st = po.init_states(cfg.width, cfg.height)
    acc = np.zeros(cfg.width * cfg.height * 4, np.float32)
    rows = list(range(3, cfg.height, cfg.height // 9))
    hit_textured = 0
    for frame, (inp, reset) in enumerate(_c5_schedule(4)):
        if reset:
            r.reset_accumulation()
            acc[:] = 0.0
        r.render(ds, cfg.spp, cfg.depth, inp, flags=abi.RT_FLAG_ACCUMULATE)
        torch.cuda.synchronize()
        # the oracle renders only the sampled rows; accumulation of the other rows is not compared
        ref, _, _ = po.render(osc, cfg.width, cfg.height, cfg.spp, cfg.depth, inp, st, accum=acc,
                              rows=(rows[0], cfg.height), row_step=rows[1] - rows[0], threads=THREADS)
        img = r.image()
        np.testing.assert_array_equal(img[rows], ref[rows], err_msg=f"frame {frame}")
        got_acc = r.accum.cpu().numpy().reshape(cfg.height, cfg.width, 4)
        np.testing.assert_array_equal(got_acc[rows], acc.reshape(cfg.height, cfg.width, 4)[rows])
        hit_textured += int(np.count_nonzero(img[rows] != img[rows][:, :1]))
    assert hit_textured > 0


def test_c3_configured_256spp_rows_match_oracle():
    cfg = scenes.CONFIGS["c3"]
    assert (cfg.width, cfg.height, cfg.spp, cfg.depth) == (3840, 2160, 256, 16)
    sc = scenes.builtin(cfg.scene)
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    r.render(DeviceScene(sc), cfg.spp, cfg.depth, cfg.inputs())
    torch.cuda.synchronize()
    st = po.init_states(cfg.width, cfg.height)
    step = cfg.height // 12
    rows = list(range(5, cfg.height, step))
    ref, _, _ = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st,
                          rows=(5, cfg.height), row_step=step, threads=THREADS)
    np.testing.assert_array_equal(r.image()[rows], ref[rows])
    np.testing.assert_array_equal(r.states().reshape(cfg.height, cfg.width, -1)[rows, :, :6],
                                  st.reshape(cfg.height, cfg.width, -1)[rows, :, :6])


@pytest.mark.parametrize("variant", [2, 3, 4])
def test_image_texture_without_image_is_cyan(variant):
    """RT_IMAGE albedo with image = -1 in a scene with no images: Image::value's data == nullptr branch
    (Texture.cuh:83-84) returns cyan; the kernel must not index the (absent) image table."""
    from cudaraytracer_amd._lib import lib
    lib().rt_set_variant(variant)
    try:
        cfg = scenes.CONFIGS["c5"].scaled(96, 64, 2)
        sc = scenes.builtin(cfg.scene)
        for i in range(len(sc.materials)):
            if sc.materials[i].albedo.type == abi.RT_IMAGE:
                sc.materials[i].albedo.image = -1
        sc.images = []
        r = Renderer(cfg.width, cfg.height)
        r.render_init()
        r.render(DeviceScene(sc), cfg.spp, cfg.depth, cfg.inputs())
        torch.cuda.synchronize()
        st = po.init_states(cfg.width, cfg.height)
        ref, _, _ = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st)
        np.testing.assert_array_equal(r.image(), ref)
    finally:
        lib().rt_set_variant(-1)


@pytest.mark.parametrize("layout", [3, 4])
def test_texel_layouts_give_the_same_image(layout, c5_scene):
    """RGB8 (the reference's 3-byte texels) and RGBA8-padded device layouts render identical images."""
    from cudaraytracer_amd._lib import lib
    cfg = scenes.CONFIGS["c5"].scaled(160, 96, 2)
    prev = lib().rt_set_tuning(6, layout)
    try:
        ds = DeviceScene(c5_scene)
    finally:
        lib().rt_set_tuning(6, prev)
    assert ds.info().device_bytes >= 3 * 8192 * 4096 * layout
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs())
    torch.cuda.synchronize()
    st = po.init_states(cfg.width, cfg.height)
    ref, _, _ = po.render(po.OracleScene(c5_scene), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st)
    np.testing.assert_array_equal(r.image(), ref)
