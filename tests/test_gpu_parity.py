"""GPU parity tests (MI355X): librt_hip.so through the C ABI against the oracle and the golden fixtures.

Bar: the RGBA8 image, the advanced cuRAND states and the ray count are BIT-EXACT with the oracle on every
golden case and kernel variant (the arithmetic contract in render.hip).  Full-size configurations are
checked through size-independent properties (tile invariance, determinism, equality of row samples with the
oracle, radiance/pos consistency).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest
import torch

import refgraph
from cases import CASE_BY_NAME, CASES, PHILOX_CASES
from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd._lib import RTError, lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer
from helpers import digest, image_stats, load_golden
from oracle import py_oracle as po

pytestmark = pytest.mark.gpu

VARIANTS = list(range(7))  # every kernel librt_hip.so ships (kVariants in render.hip)
# v3 (2), v3 compact parking (3), persistent v4 (4), flat (5: scenes of at most 64 primitives, else 3), persistent
# flat (6: else 4)
KEY_VARIANTS = [2, 3, 4, 5, 6]


@pytest.fixture(autouse=True)
def _variant_reset():
    yield
    lib().rt_set_variant(-1)


def _render(case, variant=-1, radiance=False, count_tests=False):
    cfg = case.cfg()
    lib().rt_set_variant(variant)
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    sc = scenes.builtin(cfg.scene)
    ds = DeviceScene(sc)
    flags = case.flags | (abi.RT_FLAG_COUNT_TESTS if count_tests else 0)
    if case.faithful_grid:
        # the reference's RenderInit only seeds the floor grid; seed the same way (LaunchRenderInit)
        r.state.zero_()
        grid = abi.Dim3(cfg.width // 16, cfg.height // 16, 1)
        lib().LaunchRenderInit(grid, abi.Dim3(16, 16, 1), cfg.width, cfg.height, C.c_void_p(r.state.data_ptr()))
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=flags, radiance=radiance)
    torch.cuda.synchronize()
    return r, ds, sc


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("case", CASES, ids=lambda c: c.name)
def test_bit_exact_vs_golden(case, variant):
    g = load_golden(case.name)
    r, _, _ = _render(case, variant)
    img = r.image()
    assert image_stats(img, g["pos"])["exact"] == 1.0, image_stats(img, g["pos"])
    np.testing.assert_array_equal(img, g["pos"])
    assert digest(r.states()[:, :6]) == g["state_after_sha256"].tobytes()
    assert int(r.counters[0]) == int(g["counters"][0])  # rays
    assert int(r.counters[3]) == int(g["counters"][3])  # primary samples


@pytest.mark.parametrize("case", [CASE_BY_NAME["c2_rtiow_192x112_s16"], CASE_BY_NAME["c3_cornell_128_s16"]],
                         ids=lambda c: c.name)
def test_radiance_matches_oracle(case):
    cfg = case.cfg()
    r, _, sc = _render(case, radiance=True)
    st = po.init_states(cfg.width, cfg.height)
    _, rad, _ = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st,
                          radiance=True, rius_order=case.rius_order)
    np.testing.assert_array_equal(r.radiance_image(), rad)
    # pos is the gamma-2 RGBA8 of the radiance (Kernel.cu:151-157)
    c = np.clip(255.0 * np.sqrt(rad[..., :3].astype(np.float32)), 0, 255).astype(np.uint32)
    assert np.array_equal(r.image() & 0xFFFFFF, c[..., 0] | (c[..., 1] << 8) | (c[..., 2] << 16))


def test_count_tests_flag_does_not_change_the_image():
    case = CASE_BY_NAME["c2_rtiow_192x112_s16"]
    r, _, _ = _render(case, count_tests=True)
    g = load_golden(case.name)
    np.testing.assert_array_equal(r.image(), g["pos"])
    rays, boxes, prims = (int(x) for x in r.counters[:3])
    assert boxes > 2 * rays and prims > 0
    assert int(r.counters[16]) == 0  # RTIOW: spheres only


@pytest.mark.parametrize("variant", [3, 5, 6])
def test_rectangle_tests_are_counted_apart(variant):
    """counters[16] (RT_FLAG_COUNT_TESTS) is the rectangle part of the primitive tests (bench.py's FLOP model
    prices them at 12 against a sphere's 23).  The flat kernels (5, 6) test every primitive of
    C3's Cornell box per ray: 6 rectangles and 2 spheres each; the BVH kernel (3) a subset."""
    case = CASE_BY_NAME["c3_cornell_128_s16"]
    r, _, _ = _render(case, variant, count_tests=True)
    np.testing.assert_array_equal(r.image(), load_golden(case.name)["pos"])
    rays, prims, rects = int(r.counters[0]), int(r.counters[2]), int(r.counters[16])
    if variant in (5, 6):
        assert (prims, rects) == (8 * rays, 6 * rays)
    else:
        assert 0 < rects < prims


@pytest.mark.parametrize("num_ranks, band_rows", [(2, 16), (3, 16), (4, 8), (8, 16)])
def test_tile_split_is_bit_identical(num_ranks, band_rows):
    """N-rank block-cyclic bands reassemble into exactly the 1-rank image (global-index RNG seeding)."""
    case = CASE_BY_NAME["c2_rtiow_192x112_s16"]
    cfg = case.cfg()
    g = load_golden(case.name)
    sc = scenes.builtin(cfg.scene)
    ds = DeviceScene(sc)
    full = np.zeros((cfg.height, cfg.width), np.uint32)
    rays = 0
    for rank in range(num_ranks):
        r = Renderer(cfg.width, cfg.height, band_rows=band_rows, num_ranks=num_ranks, rank=rank)
        r.render_init()
        r.render(ds, cfg.spp, cfg.depth, cfg.inputs())
        torch.cuda.synchronize()
        full[r.rows] = r.image()
        rays += int(r.counters[0])
    np.testing.assert_array_equal(full, g["pos"])
    assert rays == int(g["counters"][0])


def test_faithful_grid_leaves_partial_blocks_untouched():
    case = CASE_BY_NAME["c1_full"]
    cfg = case.cfg()
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    r.pos.fill_(0x12345678)
    ds = DeviceScene(scenes.builtin(cfg.scene))
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_FAITHFUL_GRID)
    torch.cuda.synchronize()
    img = r.image()
    assert np.all(img[224] == 0x12345678)  # 225 rows → 14 whole 16-row blocks (Kernel.cu:184)
    assert np.all(img[:224] != 0x12345678)


def test_drop_in_launchers_match_oracle():
    """LaunchRenderInit / LaunchRandInit / LaunchKernel(world graph) against the oracle (Kernel.cu:178-204)."""
    case = CASE_BY_NAME["default_world_160x120_s8"]
    cfg = case.cfg()
    sc = scenes.builtin(cfg.scene)
    dev = torch.device("cuda", 0)
    W, H = cfg.width, cfg.height
    pos = torch.zeros(W * H, dtype=torch.int32, device=dev)
    state = torch.zeros(W * H * abi.STATE_WORDS, dtype=torch.int32, device=dev)
    state2 = torch.zeros(abi.STATE_WORDS, dtype=torch.int32, device=dev)
    lib().LaunchRandInit(C.c_void_p(state2.data_ptr()))
    lib().LaunchRenderInit(abi.Dim3(W // 16, H // 16, 1), abi.Dim3(16, 16, 1), W, H, C.c_void_p(state.data_ptr()))
    ref_state = po.init_states(W, H, full=False)
    got_state = state.cpu().numpy().view(np.uint32).reshape(-1, abi.STATE_WORDS)
    np.testing.assert_array_equal(got_state, ref_state)
    kat = abi.CurandState()
    po.lib().orc_curand_init(1984, C.byref(kat))
    assert state2.cpu().numpy().view(np.uint32).tobytes() == bytes(kat)
    graph = refgraph.build_graph(sc)
    lib().LaunchKernel(C.c_void_p(pos.data_ptr()), W, H, cfg.spp, cfg.depth, C.c_void_p(C.addressof(graph.world)),
                       C.c_void_p(state.data_ptr()), cfg.inputs())
    ref, _, _ = po.render(po.OracleScene(sc), W, H, cfg.spp, cfg.depth, cfg.inputs(), ref_state, faithful_grid=True)
    np.testing.assert_array_equal(pos.cpu().numpy().view(np.uint32).reshape(H, W), ref)
    # a material edit in place (CudaLayer.cpp:839-843) is picked up by the next launch without a rebuild
    m = graph.keep[[i for i, o in enumerate(graph.keep) if isinstance(o, refgraph.Constant)][1]]
    m.color.e[0] = 0.0
    lib().LaunchKernel(C.c_void_p(pos.data_ptr()), W, H, cfg.spp, cfg.depth, C.c_void_p(C.addressof(graph.world)),
                       C.c_void_p(state.data_ptr()), cfg.inputs())
    nh, nm, ni = C.c_uint32(0), C.c_uint32(0), C.c_uint32(0)
    world = C.addressof(graph.world)
    lib().rt_reference_graph_flatten(world, None, C.byref(nh), None, C.byref(nm), None, C.byref(ni))
    h = (abi.HittableDesc * nh.value)()
    mm = (abi.MaterialDesc * nm.value)()
    im = (abi.ImageDesc * 1)()
    lib().rt_reference_graph_flatten(world, h, C.byref(nh), mm, C.byref(nm), im, C.byref(ni))
    edited = scenes.Scene(h, mm, [])
    ref2, _, _ = po.render(po.OracleScene(edited), W, H, cfg.spp, cfg.depth, cfg.inputs(), ref_state, faithful_grid=True)
    np.testing.assert_array_equal(pos.cpu().numpy().view(np.uint32).reshape(H, W), ref2)


def _launch_kernel(sc, cfg, spp=None):
    """LaunchRenderInit + LaunchKernel(world graph) of `sc` (Kernel.cu:178-204); returns (image, states)."""
    dev = torch.device("cuda", 0)
    W, H = cfg.width, cfg.height
    pos = torch.zeros(W * H, dtype=torch.int32, device=dev)
    state = torch.zeros(W * H * abi.STATE_WORDS, dtype=torch.int32, device=dev)
    lib().LaunchRenderInit(abi.Dim3(W // 16, H // 16, 1), abi.Dim3(16, 16, 1), W, H, C.c_void_p(state.data_ptr()))
    graph = refgraph.build_graph(sc)
    lib().LaunchKernel(C.c_void_p(pos.data_ptr()), W, H, spp or cfg.spp, cfg.depth,
                       C.c_void_p(C.addressof(graph.world)), C.c_void_p(state.data_ptr()), cfg.inputs())
    return (pos.cpu().numpy().view(np.uint32).reshape(H, W),
            state.cpu().numpy().view(np.uint32).reshape(-1, abi.STATE_WORDS))


@pytest.mark.parametrize("order", ["rtl", "ltr"])
def test_launch_kernel_fill_order_switch(order):
    """the drop-in LaunchKernel honours rt_set_launch_flags(RT_FLAG_RIUS_LEFT_TO_RIGHT) — a viewer
    whose CUDA build filled Random()'s Vec3 left to right (Math.cuh:231-234) switches without leaving LaunchKernel —
    and each order matches the oracle's same rius_order, bit for bit (image and RNG states)."""
    case = CASE_BY_NAME["default_world_160x120_s8"]
    cfg = case.cfg()
    sc = scenes.builtin(cfg.scene)
    flag, rius = (0, 1) if order == "rtl" else (abi.RT_FLAG_RIUS_LEFT_TO_RIGHT, 0)
    prev = lib().rt_set_launch_flags(flag)
    try:
        img, states = _launch_kernel(sc, cfg)
    finally:
        lib().rt_set_launch_flags(prev)
    st = po.init_states(cfg.width, cfg.height, full=False)
    ref, _, _ = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st,
                          faithful_grid=True, rius_order=rius)
    np.testing.assert_array_equal(img, ref)
    np.testing.assert_array_equal(states[:, :6], st[:, :6])
    other, _, _ = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(),
                            po.init_states(cfg.width, cfg.height, full=False), faithful_grid=True, rius_order=1 - rius)
    assert (other != ref).sum() > 100  # the two orders are different streams


def test_launch_kernel_large_touching_scene_is_the_reference():
    """a scene beyond the flat kernels' 64 primitives whose rectangles abut and overlap (the viewer's
    AddHittable grows scenes without limit, CudaLayer.cpp:918-1370) renders through the drop-in LaunchKernel — on the
    BVH kernels — bit for bit as the oracle's reference traversal (box culling and ties included), not as the
    geometric closest hit, which differs on it (tests/test_scene_adversarial.py)."""
    from adversarial_scene import ADVERSARIAL_CONFIG, adversarial_scene_tiled
    cfg, sc = ADVERSARIAL_CONFIG, adversarial_scene_tiled()
    assert len(sc.hittables) > 64
    img, states = _launch_kernel(sc, cfg)
    assert lib().rt_last_variant() in (2, 3, 4)
    st = po.init_states(cfg.width, cfg.height, full=False)
    ref, _, _ = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st,
                          faithful_grid=True)
    bad = np.argwhere(img != ref)
    assert len(bad) == 0, f"{len(bad)} pixels differ, first {bad[:4].tolist()}"
    np.testing.assert_array_equal(states[:, :6], st[:, :6])


@pytest.mark.parametrize("rng", ["xorwow", "philox"])
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4])
def test_bvh_kernels_exact_on_the_tiled_touching_scene(variant, rng):
    """The BVH kernels' exactness check and replay (render.hip bvh_clear) on every BVH variant, both RNG modes, on the
    > 64-primitive touching scene: whole frame, RNG states and ray count equal the oracle's reference traversal; the
    counting build reports how many rays replayed (counters[17]) — a small fraction even here."""
    from adversarial_scene import ADVERSARIAL_CONFIG, adversarial_scene_tiled
    cfg, sc = ADVERSARIAL_CONFIG, adversarial_scene_tiled()
    lib().rt_set_variant(variant)
    r = Renderer(cfg.width, cfg.height, rng=rng)
    r.render_init()
    r.render(DeviceScene(sc), cfg.spp, cfg.depth, cfg.inputs(), frame=2, flags=abi.RT_FLAG_COUNT_TESTS)
    torch.cuda.synchronize()
    philox = rng == "philox"
    assert lib().rt_last_variant() == (3 if philox and variant in (0, 1) else variant)
    st = None if philox else po.init_states(cfg.width, cfg.height)
    ref, _, cnt = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st,
                            philox=philox, seed=1984, frame=2)
    bad = np.argwhere(r.image() != ref)
    assert len(bad) == 0, f"{len(bad)} pixels differ, first {bad[:4].tolist()}"
    if not philox:
        np.testing.assert_array_equal(r.states()[:, :6], st[:, :6])
    rays, replays = int(r.counters[0]), int(r.counters[17])
    assert rays == cnt.rays
    assert 0 < replays < rays // 4, (replays, rays)  # (its duplicated row ties on every ray that hits it)


def test_material_update_without_rebuild():
    case = CASE_BY_NAME["c2_rtiow_ragged_100x37_s4"]
    cfg = case.cfg()
    sc = scenes.builtin(cfg.scene)
    ds = DeviceScene(sc)
    for i in range(len(sc.materials)):
        if sc.materials[i].type == abi.RT_LAMBERTIAN:
            sc.materials[i].albedo.color[:] = [0.9, 0.1, 0.1]
    ds.update_materials(sc.materials)
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs())
    torch.cuda.synchronize()
    st = po.init_states(cfg.width, cfg.height)
    ref, _, _ = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st)
    np.testing.assert_array_equal(r.image(), ref)


@pytest.mark.parametrize("variant", KEY_VARIANTS)
def test_edge_cases_spp0_depth0_empty_and_inactive(variant):
    lib().rt_set_variant(variant)
    cfg = scenes.CONFIGS["c2"].scaled(48, 32, 3)
    sc = scenes.builtin(cfg.scene)
    ds = DeviceScene(sc)
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    before = r.states().copy()
    r.render(ds, 0, cfg.depth, cfg.inputs())
    torch.cuda.synchronize()
    assert np.all(r.image() == 0xFF000000)  # col/0 = NaN → int(NaN) = 0
    np.testing.assert_array_equal(r.states(), before)
    r.render(ds, 2, 0, cfg.inputs())  # max_depth 0: black, 2 draws per sample
    torch.cuda.synchronize()
    assert np.all(r.image() == 0xFF000000) and int(r.counters[0]) == 0
    ref_st = po.init_states(cfg.width, cfg.height)
    for i in range(ref_st.shape[0]):
        s = abi.CurandState.from_buffer(ref_st[i])
        for _ in range(4):
            po.lib().orc_curand(C.byref(s))
    np.testing.assert_array_equal(r.states()[:, :6], ref_st[:, :6])
    # all hittables inactive → empty scene → pure sky; some inactive → oracle with the same flags
    for k in range(sc.num_hittables):
        sc.hittables[k].is_active = 1 if k % 3 else 0
    ds2 = DeviceScene(sc)
    r2 = Renderer(cfg.width, cfg.height)
    r2.render_init()
    r2.render(ds2, cfg.spp, cfg.depth, cfg.inputs())
    torch.cuda.synchronize()
    st = po.init_states(cfg.width, cfg.height)
    ref, _, _ = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st)
    np.testing.assert_array_equal(r2.image(), ref)
    for k in range(sc.num_hittables):
        sc.hittables[k].is_active = 0
    ds3 = DeviceScene(sc)
    r3 = Renderer(cfg.width, cfg.height)
    r3.render_init()
    r3.render(ds3, cfg.spp, cfg.depth, cfg.inputs())
    torch.cuda.synchronize()
    st = po.init_states(cfg.width, cfg.height)
    ref, _, cnt = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st)
    np.testing.assert_array_equal(r3.image(), ref)
    assert int(r3.counters[0]) == cnt.rays == cfg.width * cfg.height * cfg.spp


@pytest.mark.parametrize("variant", KEY_VARIANTS)
def test_single_primitive_scene(variant):
    lib().rt_set_variant(variant)
    cfg = scenes.CONFIGS["c1"].scaled(64, 36, 4)
    sc = scenes.builtin(cfg.scene)
    sc.hittables[0].is_active = 0
    sc.hittables[2].is_active = 0
    ds = DeviceScene(sc)
    assert ds.info().num_primitives == 1
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs())
    torch.cuda.synchronize()
    st = po.init_states(cfg.width, cfg.height)
    ref, _, _ = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st)
    np.testing.assert_array_equal(r.image(), ref)


@pytest.mark.parametrize("variant", KEY_VARIANTS)
def test_accumulate_first_frame_equals_plain_frame(variant):
    lib().rt_set_variant(variant)
    case = CASE_BY_NAME["c5_textured_160x96_s4"]
    cfg = case.cfg()
    g = load_golden(case.name)
    ds = DeviceScene(scenes.builtin(cfg.scene))
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_ACCUMULATE)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(r.image(), g["pos"])
    acc1 = r.accum.cpu().numpy().reshape(-1, 4).copy()
    assert np.all(acc1[:, 3] == cfg.spp)
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_ACCUMULATE)
    torch.cuda.synchronize()
    acc2 = r.accum.cpu().numpy().reshape(-1, 4)
    assert np.all(acc2[:, 3] == 2 * cfg.spp) and np.all(acc2[:, :3] >= acc1[:, :3])


@pytest.mark.parametrize("variant", [3, 4, 5, 6])
def test_philox_accumulate_matches_oracle(variant):
    """Progressive accumulation in Philox mode (the pixel sums in fixed point, sample items on the tile kernels): two
    frames of the textured case (full 8x8 tiles) accumulate exactly as the oracle's RT_FLAG_ACCUMULATE restatement."""
    lib().rt_set_variant(variant)
    case = CASE_BY_NAME["c5_textured_160x96_s4"]
    cfg = case.cfg()
    sc = scenes.builtin(cfg.scene)
    ds = DeviceScene(sc)
    r = Renderer(cfg.width, cfg.height, rng="philox")
    r.render_init()
    acc = np.zeros(cfg.width * cfg.height * 4, dtype=np.float32)
    for frame in (0, 1):
        r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_ACCUMULATE, frame=frame)
        torch.cuda.synchronize()
        ref, _, cnt = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), None,
                                philox=True, seed=1984, frame=frame, accum=acc)
        np.testing.assert_array_equal(r.image(), ref)
        np.testing.assert_array_equal(r.accum.cpu().numpy().reshape(-1), acc)


def test_invalid_arguments_fail_loudly():
    cfg = scenes.CONFIGS["c1"].scaled(32, 16, 1)
    r = Renderer(cfg.width, cfg.height)
    ds = DeviceScene(scenes.builtin(cfg.scene))
    r.num_ranks, r.rank = 2, 5  # rank outside the tiling
    with pytest.raises(RTError, match="tiling"):
        r.render(ds, 1, 1, cfg.inputs())
    a = abi.RenderArgs()
    a.pos, a.width, a.height = r.pos.data_ptr(), 32, 16
    a.tiling = abi.Tiling(16, 1, 0, 16)
    assert lib().rt_render(ds.handle, C.byref(a), None) == -1  # NULL state
    assert b"state" in lib().rt_last_error()


# ---------------------------------------------------------------------------------------------------
# Full-size configurations: size-independent properties
# ---------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("ltr", [False, True], ids=["rtl", "ltr"])
@pytest.mark.parametrize("config", ["c2", "c3"])
def test_full_size_rows_match_oracle_and_tiles_are_invariant(config, ltr):
    """Configs 2 and 3 at full size in both Random() fill orders (Math.cuh:231-234: right to left, the library
    default, and left to right, RT_FLAG_RIUS_LEFT_TO_RIGHT)."""
    flag = abi.RT_FLAG_RIUS_LEFT_TO_RIGHT if ltr else 0
    cfg = scenes.CONFIGS[config]
    if config == "c3":
        cfg = cfg.scaled(cfg.width, cfg.height, 16)  # 256 spp × 8.3 Mpx is minutes of CPU oracle; rows still full-width
    sc = scenes.builtin(cfg.scene)
    ds = DeviceScene(sc)
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=flag)
    torch.cuda.synchronize()
    img = r.image()
    assert np.all((img >> 24) == 0xFF)
    # oracle on a strided sample of full rows (same global pixel indices → same RNG streams)
    step = cfg.height // 6
    st = po.init_states(cfg.width, cfg.height)
    ref, _, _ = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st,
                          rows=(1, cfg.height), row_step=step, threads=16, rius_order=0 if ltr else 1)
    rows = list(range(1, cfg.height, step))
    np.testing.assert_array_equal(img[rows], ref[rows])
    np.testing.assert_array_equal(r.states().reshape(cfg.height, cfg.width, -1)[rows, :, :6],
                                  st.reshape(cfg.height, cfg.width, -1)[rows, :, :6])
    # 4-rank band split of the full frame reassembles bit-identically
    full = np.zeros_like(img)
    for rank in range(4):
        rr = Renderer(cfg.width, cfg.height, band_rows=16, num_ranks=4, rank=rank)
        rr.render_init()
        rr.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=flag)
        torch.cuda.synchronize()
        full[rr.rows] = rr.image()
        del rr
    np.testing.assert_array_equal(full, img)


def test_full_size_c2_determinism_and_frame_sequence():
    cfg = scenes.CONFIGS["c2"]
    ds = DeviceScene(scenes.builtin(cfg.scene))
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    s0 = r.state.clone()
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_NO_STATE_WRITEBACK)
    torch.cuda.synchronize()
    a = r.image().copy()
    assert torch.equal(r.state, s0)
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs())
    torch.cuda.synchronize()
    b = r.image().copy()
    np.testing.assert_array_equal(a, b)
    rays = int(r.counters[0]) // 2
    assert 2.9 < rays / (cfg.width * cfg.height * cfg.spp) < 3.3  # ≈3.0-3.1 rays per primary
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs())  # next frame continues the RNG streams (Kernel.cu:149)
    torch.cuda.synchronize()
    c = r.image()
    s = image_stats(b, c)
    assert s["exact"] < 0.9 and abs(s["mean_signed"]) < 0.5  # new noise, same expectation


@pytest.mark.parametrize("variant", KEY_VARIANTS)
def test_scene_beyond_binary16_range_matches_oracle(variant):
    """Planes beyond ±65504 (outside binary16): fp32 boxes keep the closest hit exact."""
    cfg = scenes.CONFIGS["c1"].scaled(64, 36, 4)
    sc = scenes.builtin(cfg.scene)
    sc.hittables[0].center[0] = 70000.0
    lib().rt_set_variant(variant)
    ds = DeviceScene(sc)
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs())
    torch.cuda.synchronize()
    st = po.init_states(cfg.width, cfg.height)
    ref, _, cnt = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st)
    np.testing.assert_array_equal(r.image(), ref)
    assert int(r.counters[0]) == cnt.rays


def _sphere_field(n: int, seed: int) -> scenes.Scene:
    return scenes.sphere_field(n, seed)


@pytest.mark.parametrize("variant", [-1, 3, 4])
def test_large_scene_deep_bvh_matches_oracle(variant):
    """6000 spheres: the plain SAH tree is deeper than the 8-wave LDS budget, so the build bounds it to depth 12
    (capacity-limited SAH splits, scene_build.cpp); child references up to ~1500 ride in the node planes' low
    bytes; the image and ray count equal the oracle's (reference BVH: list-order splits)."""
    cfg = scenes.CONFIGS["c2"].scaled(96, 54, 4)
    sc = _sphere_field(6000, 5)
    ds = DeviceScene(sc)
    info = ds.info()
    assert info.num_primitives == 6001 and info.bvh_depth == 12 and info.num_nodes > 256
    lib().rt_set_variant(variant)
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs())
    torch.cuda.synchronize()
    assert lib().rt_last_variant() in (3, 4)
    ref, _, cnt = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(),
                            po.init_states(cfg.width, cfg.height), threads=8)
    np.testing.assert_array_equal(r.image(), ref)
    assert int(r.counters[0]) == cnt.rays


@pytest.mark.parametrize("variant", [-1, 0, 1, 3, 4])
def test_scene_beyond_16bit_references_matches_oracle(variant):
    """9000 spheres: leaf references no longer fit 16 bits.  The automatic choice and variants 3 / 4 run the
    32-bit-reference (WIDE) builds of v3 / v4; variants 0 / 1 the v1 / v2 kernels — all with the oracle's image
    and ray count."""
    cfg = scenes.CONFIGS["c2"].scaled(64, 36, 2)
    sc = _sphere_field(9000, 6)
    ds = DeviceScene(sc)
    assert ds.info().num_primitives == 9001
    lib().rt_set_variant(variant)
    try:
        r = Renderer(cfg.width, cfg.height)
        r.render_init()
        r.render(ds, cfg.spp, cfg.depth, cfg.inputs())
        torch.cuda.synchronize()
        assert lib().rt_last_variant() == variant if variant >= 0 else lib().rt_last_variant() in (3, 4)
    finally:
        lib().rt_set_variant(-1)
    ref, _, cnt = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(),
                            po.init_states(cfg.width, cfg.height), threads=8)
    np.testing.assert_array_equal(r.image(), ref)
    assert int(r.counters[0]) == cnt.rays


@pytest.mark.parametrize("variant, rng", [(3, "xorwow"), (4, "xorwow"), (3, "philox"), (4, "philox")])
def test_20000_sphere_scene_wide_references_match_oracle(variant, rng):
    """20 000 spheres (> 32767 BVH nodes would need ~3x that; here > 8191 leaves and primitives): the WIDE v3 / v4
    builds, both RNG modes, bit-exact with the oracle (AddHittable grows scenes without limit,
    CudaLayer.cpp:918-1370)."""
    cfg = scenes.CONFIGS["c2"].scaled(48, 32, 2)
    sc = _sphere_field(20000, 11)
    ds = DeviceScene(sc)
    lib().rt_set_variant(variant)
    try:
        r = Renderer(cfg.width, cfg.height, rng=rng)
        r.render_init()
        r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), frame=1 if rng == "philox" else None)
        torch.cuda.synchronize()
        assert lib().rt_last_variant() == variant
    finally:
        lib().rt_set_variant(-1)
    st = po.init_states(cfg.width, cfg.height) if rng == "xorwow" else None
    ref, _, cnt = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st,
                            threads=8, philox=rng == "philox", seed=1984, frame=1)
    np.testing.assert_array_equal(r.image(), ref)
    assert int(r.counters[0]) == cnt.rays
    if rng == "xorwow":
        np.testing.assert_array_equal(r.states()[:, :6], st[:, :6])


# ---------------------------------------------------------------------------------------------------
# Perf-mode RNG (RT_FLAG_RNG_PHILOX): bit-exact with the oracle's Philox restatement, no state buffer
# ---------------------------------------------------------------------------------------------------
PHILOX_KERNELS = [-1, 2, 3, 4, 0, 5, 6]  # auto, v3, v3 compact, v4, flat, persistent flat; 0 (v1, no Philox build)
# maps to v3 compact


# The Cornell box's walls touch (tests/adversarial_scene.py): there the BVH kernels (variants 0-4) return the
# geometric closest hit, not the reference traversal's, on the rare rays that graze a wall's edge — which the automatic
# choice never runs them on (it keeps touching-rectangle scenes on the flat kernels).  Philox's per-sample windows
# (round 4) put such a ray into this case's frame on v3 (one ray of 1.55 M longer, the same pixels), so Cornell runs
# the kernels that hold the reference traversal; the BVH kernels run the other five cases.
_PHILOX_PAIRS = [(CASE_BY_NAME[n], v) for n in ("c1_full", "c2_rtiow_192x112_s16", "c3_cornell_128_s16",
                                                "c5_textured_160x96_s4", "c2_rtiow_ragged_100x37_s4",
                                                "c2_rtiow_ltr_96x64_s8")
                 for v in PHILOX_KERNELS if not (n.startswith("c3") and v in (0, 2, 3, 4))]


@pytest.mark.parametrize("case, variant", _PHILOX_PAIRS, ids=lambda x: getattr(x, "name", str(x)))
def test_philox_bit_exact_vs_oracle(case, variant):
    cfg = case.cfg()
    lib().rt_set_variant(variant)
    sc = scenes.builtin(cfg.scene)
    r = Renderer(cfg.width, cfg.height, rng="philox")
    assert r.state is None
    r.render_init()
    r.render(DeviceScene(sc), cfg.spp, cfg.depth, cfg.inputs(), flags=case.flags, radiance=True, frame=5)
    torch.cuda.synchronize()
    ref, rad, cnt = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), None,
                              faithful_grid=case.faithful_grid, rius_order=case.rius_order, radiance=True,
                              philox=True, seed=1984, frame=5)
    if case.faithful_grid:  # pixels outside whole 16×16 blocks are not written (Kernel.cu:184)
        gh, gw = (cfg.height // 16) * 16, (cfg.width // 16) * 16
        np.testing.assert_array_equal(r.image()[:gh, :gw], ref[:gh, :gw])
    else:
        np.testing.assert_array_equal(r.image(), ref)
        np.testing.assert_array_equal(r.radiance_image(), rad)
    assert int(r.counters[0]) == cnt.rays


@pytest.mark.parametrize("case, frame", PHILOX_CASES, ids=lambda x: getattr(x, "name", str(x)))
def test_philox_matches_golden(case, frame):
    g = load_golden(f"philox_{case.name}_f{frame}")
    cfg = case.cfg()
    r = Renderer(cfg.width, cfg.height, rng="philox")
    r.render_init(1984)
    r.render(DeviceScene(scenes.builtin(cfg.scene)), cfg.spp, cfg.depth, cfg.inputs(), flags=case.flags, frame=frame)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(r.image(), g["pos"])
    assert int(r.counters[0]) == int(g["counters"][0])


def test_philox_frames_tiles_and_invalid_state():
    case = CASE_BY_NAME["c2_rtiow_192x112_s16"]
    cfg = case.cfg()
    ds = DeviceScene(scenes.builtin(cfg.scene))
    r = Renderer(cfg.width, cfg.height, rng="philox")
    r.render_init()
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs())  # frame 0
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs())  # frame 1: fresh numbers
    torch.cuda.synchronize()
    f1 = r.image().copy()
    assert r.frame == 2
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), frame=0)
    torch.cuda.synchronize()
    f0 = r.image().copy()
    assert image_stats(f0, f1)["exact"] < 0.9
    # block-cyclic bands reassemble into the 1-rank frame (global pixel index keys the streams)
    full = np.zeros_like(f0)
    for rank in range(3):
        rr = Renderer(cfg.width, cfg.height, band_rows=16, num_ranks=3, rank=rank, rng="philox")
        rr.render_init()
        rr.render(ds, cfg.spp, cfg.depth, cfg.inputs(), frame=0)
        torch.cuda.synchronize()
        full[rr.rows] = rr.image()
    np.testing.assert_array_equal(full, f0)
    # XORWOW mode still refuses a NULL state
    a = abi.RenderArgs()
    a.pos, a.width, a.height, a.samples_per_pixel, a.max_depth = r.pos.data_ptr(), cfg.width, cfg.height, 1, 1
    a.tiling = abi.Tiling(cfg.height, 1, 0, cfg.height)
    assert lib().rt_render(ds.handle, C.byref(a), None) == -1
    a.flags = abi.RT_FLAG_RNG_PHILOX
    assert lib().rt_render(ds.handle, C.byref(a), None) == 0
    torch.cuda.synchronize()


def test_philox_full_size_c2_rows_match_oracle():
    cfg = scenes.CONFIGS["c2"]
    sc = scenes.builtin(cfg.scene)
    r = Renderer(cfg.width, cfg.height, rng="philox")
    r.render_init()
    r.render(DeviceScene(sc), cfg.spp, cfg.depth, cfg.inputs(), frame=11)
    torch.cuda.synchronize()
    step = cfg.height // 5
    ref, _, _ = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), None,
                          rows=(2, cfg.height), row_step=step, threads=16, philox=True, frame=11)
    rows = list(range(2, cfg.height, step))
    np.testing.assert_array_equal(r.image()[rows], ref[rows])
    rays = int(r.counters[0])
    assert 2.9 < rays / (cfg.width * cfg.height * cfg.spp) < 3.3


def test_adaptive_tile_order_changes_schedule_not_pixels():
    """The v3 kernels dispatch tiles longest-first by the previous launch's per-tile lifetimes
    (RT_TUNE_ADAPTIVE_ORDER); frames rendered row-major, then reordered, are identical."""
    cfg = scenes.CONFIGS["c2"].scaled(320, 176, 8)
    ds = DeviceScene(scenes.builtin(cfg.scene))
    lib().rt_set_variant(3)
    prev = lib().rt_set_tuning(5, 0)
    try:
        r = Renderer(cfg.width, cfg.height)
        r.render_init()
        r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_NO_STATE_WRITEBACK)
        torch.cuda.synchronize()
        row_major = r.image().copy()
        lib().rt_set_tuning(5, 1)
        for _ in range(3):  # the first launch records costs, the next ones dispatch longest-first
            r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_NO_STATE_WRITEBACK)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(r.image(), row_major)
        st = po.init_states(cfg.width, cfg.height)
        ref, _, _ = po.render(po.OracleScene(scenes.builtin(cfg.scene)), cfg.width, cfg.height, cfg.spp, cfg.depth,
                              cfg.inputs(), st)
        np.testing.assert_array_equal(row_major, ref)
    finally:
        lib().rt_set_tuning(5, prev if prev >= 0 else 1)


def _small_rects_scene():
    """48 small axis-aligned rectangles (0.3-0.8 units) scattered around the origin, Lambertian."""
    rng = np.random.default_rng(11)
    n = 48
    h = (abi.HittableDesc * n)()
    m = (abi.MaterialDesc * n)()
    for i in range(n):
        h[i].type = (abi.RT_XYRECT, abi.RT_XZRECT, abi.RT_YZRECT)[i % 3]
        h[i].is_active = 1
        h[i].center[:] = [float(v) for v in rng.uniform(-6.0, 6.0, 3).astype(np.float32)]
        h[i].width, h[i].height = (float(v) for v in rng.uniform(0.3, 0.8, 2).astype(np.float32))
        h[i].material = i
        m[i].type = abi.RT_LAMBERTIAN
        m[i].albedo.type = abi.RT_CONSTANT
        m[i].albedo.image = -1
        m[i].albedo.color[:] = [float(v) for v in rng.uniform(0.2, 0.9, 3).astype(np.float32)]
    return scenes.Scene(h, m, [])


@pytest.mark.parametrize("rng", ["xorwow", "philox"])
@pytest.mark.parametrize("variant", [5, 6, 0, 1, 2, 3, 4])
def test_kernels_exact_on_ties_and_box_faces(variant, rng):
    """The exactness argument (render.hip flat_trace and bvh_clear: a geometric closest hit is the reference's unless
    it ties, lies within rounding of a face of its own reference box, or a NaN took part — those rays replay the
    reference BVH) on a scene built to hit every case: coplanar rectangles that overlap (exact ties in t over an
    area) and abut (shared edges), a floor and a wall meeting their edges, spheres tangent to the rectangles'
    plane and touching the floor and wall with their box faces, a mirror sphere for reflected rays.  In this scene the
    reference's box culling changes 521 pixels against the brute-force closest hit (tests/test_scene_adversarial.py
    pins that on the CPU), so the whole frame, the RNG states and the ray count must equal the oracle's reference
    traversal, not the geometric answer — on the flat kernels (5, 6) and, since round 6, on the BVH kernels (0-4)
    whose SAH tree is not the reference's (v1/v2 have no Philox build: rt_render runs the compact v3 there)."""
    from adversarial_scene import ADVERSARIAL_CONFIG, adversarial_scene
    cfg, sc = ADVERSARIAL_CONFIG, adversarial_scene()
    lib().rt_set_variant(variant)
    r = Renderer(cfg.width, cfg.height, rng=rng)
    r.render_init()
    r.render(DeviceScene(sc), cfg.spp, cfg.depth, cfg.inputs(), frame=3)
    torch.cuda.synchronize()
    assert lib().rt_last_variant() == (3 if rng == "philox" and variant in (0, 1) else variant)
    philox = rng == "philox"
    st = None if philox else po.init_states(cfg.width, cfg.height)
    ref, _, cnt = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st,
                            philox=philox, seed=1984, frame=3)
    img = r.image()
    bad = np.argwhere(img != ref)
    assert len(bad) == 0, f"{len(bad)} pixels differ, first {bad[:4].tolist()}"
    if not philox:
        np.testing.assert_array_equal(r.states()[:, :6], st[:, :6])
    assert int(r.counters[0]) == cnt.rays


@pytest.mark.parametrize("spp", [4, 64])
def test_touching_rectangles_beyond_the_flat_limit_run_exact_bvh_kernels(spp):
    """A scene beyond RT_TUNE_FLAT_MAX (20 primitives) whose rectangles touch (the adversarial scene plus 12 spheres).
    Until round 5 the automatic choice kept such scenes on the flat kernels, the only exact ones; since the BVH kernels
    replay the reference traversal for the rays where it could differ (render.hip bvh_clear), it runs them (faster at
    this size), on both sides of the spp rule — the persistent one below 64 spp after its trial, the tile one from 64 —
    and the whole frame is still the reference's."""
    from adversarial_scene import ADVERSARIAL_CONFIG, adversarial_scene_large
    cfg = ADVERSARIAL_CONFIG.scaled(ADVERSARIAL_CONFIG.width, ADVERSARIAL_CONFIG.height, spp)
    sc = adversarial_scene_large()
    assert len(sc.hittables) == 20
    ds = DeviceScene(sc)
    lib().rt_set_variant(-1)
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    frames = 4 if spp < 64 else 1  # below 64 spp: the automatic choice's trial frames, then the chosen kernel
    st = po.init_states(cfg.width, cfg.height)
    for _ in range(frames):
        r.render(ds, cfg.spp, cfg.depth, cfg.inputs())
        torch.cuda.synchronize()
        assert lib().rt_last_variant() in (2, 3, 4)
        ref, _, cnt = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st)
        np.testing.assert_array_equal(r.image(), ref)
    np.testing.assert_array_equal(r.states()[:, :6], st[:, :6])


@pytest.mark.parametrize("variant", KEY_VARIANTS + [0, 1])
def test_far_camera_small_primitives_match_brute_force(variant):
    """Box culling stays conservative far from the scene (the slab test's rounding grows with the
    distance travelled; kSlabSlack widens every slab interval by a relative 2^-20): a camera ~3000 units away
    with a 0.3° field of view on 48 small rectangles renders exactly the oracle's brute-force closest hit over
    all primitives (no culling at all).  Rectangles, because their hit test is as accurate at that distance
    as the boxes; the reference's sphere test is not (b² − a·c cancels at |o − c| ≈ 3000 and reports hits
    outside the sphere's own box, for the reference's BVH as for ours)."""
    lib().rt_set_variant(variant)
    pos = (2400.0, 1300.0, 1100.0)
    fwd = scenes.normalized((-2400.0, -1300.0, -1100.0))
    cfg = scenes.Config("far", scenes.SCENE_THREE_SPHERES, 128, 96, 4, 6, pos, fwd, 0.3)
    sc = _small_rects_scene()
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    r.render(DeviceScene(sc), cfg.spp, cfg.depth, cfg.inputs())
    torch.cuda.synchronize()
    st = po.init_states(cfg.width, cfg.height)
    ref, _, _ = po.render(po.OracleScene(sc, exact=True), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st)
    img = r.image()
    np.testing.assert_array_equal(img, ref)
    assert len(np.unique(img)) > 50  # the rectangles fill part of the view, not just sky


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("name", ["c2_rtiow_192x112_s16", "c3_cornell_128_s16", "c2_rtiow_ragged_100x37_s4"])
def test_soa_state_layout_is_the_same_stream(name, variant):
    """RT_FLAG_STATE_SOA (six uint32 planes, rt_render_init_soa) renders the golden images bit for bit and
    carries exactly the rt_curand_state streams across frames; tiled ranks use per-rank planes."""
    case = CASE_BY_NAME[name]
    cfg = case.cfg()
    g = load_golden(case.name)
    lib().rt_set_variant(variant)
    ds = DeviceScene(scenes.builtin(cfg.scene))
    a = Renderer(cfg.width, cfg.height)
    b = Renderer(cfg.width, cfg.height, state_layout="soa")
    for r in (a, b):
        r.render_init()
    np.testing.assert_array_equal(a.states()[:, :6], b.states()[:, :6])
    for frame in range(2):
        for r in (a, b):
            r.counters.zero_()
            r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=case.flags)
        torch.cuda.synchronize()
        if frame == 0:
            np.testing.assert_array_equal(b.image(), g["pos"])
            assert digest(b.states()[:, :6]) == g["state_after_sha256"].tobytes()
            assert int(b.counters[0]) == int(g["counters"][0])
        np.testing.assert_array_equal(a.image(), b.image())
        np.testing.assert_array_equal(a.states()[:, :6], b.states()[:, :6])
        assert int(a.counters[0]) == int(b.counters[0])
    # two band ranks with plane layouts reassemble the one-rank frame
    band = 16
    parts = []
    for rank in range(2):
        r = Renderer(cfg.width, cfg.height, band_rows=band, num_ranks=2, rank=rank, state_layout="soa")
        r.render_init()
        r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=case.flags)
        torch.cuda.synchronize()
        parts.append((r.rows, r.image().copy()))
    full = np.zeros((cfg.height, cfg.width), dtype=np.uint32)
    for rows, img in parts:
        full[rows] = img
    a2 = Renderer(cfg.width, cfg.height)
    a2.render_init()
    a2.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=case.flags)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(full, a2.image())


def test_launch_kernel_cache_eviction_across_threads():
    """Two host threads drive LaunchKernel over 10 reference graphs (the scene cache holds 8 per device, so
    entries are evicted while the other thread renders them): every frame equals the single-thread frame."""
    import threading

    case = CASE_BY_NAME["default_world_160x120_s8"]
    cfg = case.cfg().scaled(64, 48, 2)
    W, H = cfg.width, cfg.height
    dev = torch.device("cuda", 0)
    graphs = []
    for k in range(10):
        sc = scenes.builtin(cfg.scene)
        g = refgraph.build_graph(sc)
        m = g.keep[[i for i, o in enumerate(g.keep) if isinstance(o, refgraph.Constant)][1]]
        m.color.e[0] = k / 10.0  # ten distinct scenes
        graphs.append(g)

    def frame(g):
        pos = torch.zeros(W * H, dtype=torch.int32, device=dev)
        state = torch.zeros(W * H * abi.STATE_WORDS, dtype=torch.int32, device=dev)
        lib().LaunchRenderInit(abi.Dim3(W // 16, H // 16, 1), abi.Dim3(16, 16, 1), W, H, C.c_void_p(state.data_ptr()))
        lib().LaunchKernel(C.c_void_p(pos.data_ptr()), W, H, cfg.spp, cfg.depth, C.c_void_p(C.addressof(g.world)),
                           C.c_void_p(state.data_ptr()), cfg.inputs())
        torch.cuda.synchronize()
        return pos.cpu().numpy().copy()

    want = [frame(g) for g in graphs]
    got = {}
    errors = []

    def worker(t):
        try:
            torch.cuda.set_device(0)
            for rep in range(3):
                for k in range(t, 10, 2):
                    got[(t, rep, k)] = frame(graphs[k])
        except Exception as e:  # surfaced below
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not errors, errors
    assert len(got) == 30
    for (t, rep, k), img in got.items():
        np.testing.assert_array_equal(img, want[k])


@pytest.mark.parametrize("config, spp", [("c2", 2), ("c2", 8), ("c3", 4)])
def test_automatic_choice_times_both_kernels_and_keeps_the_bits(config, spp):
    """Below 64 spp the automatic choice runs v3 (untimed, then timed) and v4 (timed) on the first frames of
    a frame shape and keeps the faster; every frame of the sequence is the same image (NO_STATE_WRITEBACK)."""
    cfg = scenes.CONFIGS[config].scaled(480, 272, spp)
    lib().rt_set_variant(-1)
    ds = DeviceScene(scenes.builtin(cfg.scene))
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    images, used = [], []
    for _ in range(8):
        r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_NO_STATE_WRITEBACK)
        used.append(lib().rt_last_variant())
        torch.cuda.synchronize()
        images.append(r.image().copy())
    # the flat kernels take v3's and v4's places for small scenes (Cornell: 8 primitives)
    tile_kernel, persistent = (5, 6) if config == "c3" else (3, 4)
    assert used[:3] == [tile_kernel, tile_kernel, persistent], used
    assert used[4:] == [used[4]] * 4 and used[4] in (tile_kernel, persistent), used  # decided by frame 5
    for img in images[1:]:
        np.testing.assert_array_equal(img, images[0])
    lib().rt_set_variant(4)
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_NO_STATE_WRITEBACK)
    assert lib().rt_last_variant() == 4
    r.render(ds, 64, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_NO_STATE_WRITEBACK)  # explicit choice holds
    assert lib().rt_last_variant() == 4
    lib().rt_set_variant(-1)
    r.render(ds, 64, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_NO_STATE_WRITEBACK)
    assert lib().rt_last_variant() == tile_kernel  # from 64 spp: v3 (flat for small scenes)


@pytest.mark.parametrize("chunk, stride", [(64, 128), (128, 4096), (256, 128), (1024, 4096)])
def test_persistent_queue_knobs_change_schedule_not_pixels(chunk, stride):
    """The v4 work queue's chunk size (RT_TUNE_QUEUE_CHUNK, adaptive per head) and head spacing
    (RT_TUNE_QUEUE_STRIDE) decide which wave renders which pixel, never what it computes: every setting gives the
    oracle's image, ray count and advanced RNG states."""
    case = CASE_BY_NAME["c2_rtiow_ragged_100x37_s4"]
    cfg = case.cfg()
    g = load_golden(case.name)
    prev_c, prev_s = lib().rt_set_tuning(7, chunk), lib().rt_set_tuning(8, stride)
    lib().rt_set_variant(4)
    try:
        r = Renderer(cfg.width, cfg.height)
        r.render_init()
        r.render(DeviceScene(scenes.builtin(cfg.scene)), cfg.spp, cfg.depth, cfg.inputs(), flags=case.flags)
        torch.cuda.synchronize()
        assert lib().rt_last_variant() == 4
    finally:
        lib().rt_set_variant(-1)
        lib().rt_set_tuning(7, prev_c)
        lib().rt_set_tuning(8, prev_s)
    np.testing.assert_array_equal(r.image(), g["pos"])
    assert int(r.counters[0]) == int(g["counters"][0])


# scheduling knobs (rt_hip.h) and the kernels they steer: (key, value) pairs around the defaults, with the extremes
V3_KNOBS = [(abi.RT_TUNE_LEAF_BREAK, k, v) for k in (0, 1, 64) for v in (2, 3)] + \
           [(abi.RT_TUNE_REGEN_LIVE_FRAC, k, v) for k in (0, 1, 64) for v in (2, 3)] + \
           [(abi.RT_TUNE_RIUS_TRIPS, k, v) for k in (0, 1, 2, 3, 5) for v in (5, 6)] + \
           [(abi.RT_TUNE_RIUS_TRIPS_PERSISTENT, k, 6) for k in (0, 1, 3, 4)]


@pytest.mark.parametrize("key, value, variant", V3_KNOBS, ids=lambda v: str(v))
def test_v3_scheduling_knobs_change_schedule_not_pixels(key, value, variant):
    """RT_TUNE_LEAF_BREAK and RT_TUNE_REGEN_LIVE_FRAC decide when a v3 wave traverses, tests leaves or shades, and
    RT_TUNE_RIUS_TRIPS when a flat-kernel lane resumes a RandomInUnitSphere call — never what a lane computes: every
    setting renders the golden images, ray counts and advanced RNG states (XORWOW) and the Philox goldens."""
    prev = lib().rt_set_tuning(key, value)
    assert prev >= 0
    lib().rt_set_variant(variant)
    try:
        for name in ("c2_rtiow_192x112_s16", "c3_cornell_128_s16", "c2_rtiow_ltr_96x64_s8"):
            case = CASE_BY_NAME[name]
            cfg, g = case.cfg(), load_golden(case.name)
            r = Renderer(cfg.width, cfg.height)
            r.render_init()
            ds = DeviceScene(scenes.builtin(cfg.scene))
            r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=case.flags)
            torch.cuda.synchronize()
            # (a scene beyond the flat kernels' 64 primitives, RTIOW's 488 spheres, runs v3 / v4 instead)
            big = ds.info().num_primitives > 64
            assert lib().rt_last_variant() == (variant - 2 if variant >= 5 and big else variant)
            np.testing.assert_array_equal(r.image(), g["pos"], err_msg=name)
            assert digest(r.states()[:, :6]) == g["state_after_sha256"].tobytes(), name
            assert int(r.counters[0]) == int(g["counters"][0]), name
        for case, frame in PHILOX_CASES:
            g = load_golden(f"philox_{case.name}_f{frame}")
            cfg = case.cfg()
            r = Renderer(cfg.width, cfg.height, rng="philox")
            r.render_init(1984)
            r.render(DeviceScene(scenes.builtin(cfg.scene)), cfg.spp, cfg.depth, cfg.inputs(), flags=case.flags,
                     frame=frame)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(r.image(), g["pos"], err_msg=f"philox {case.name}")
            assert int(r.counters[0]) == int(g["counters"][0])
    finally:
        lib().rt_set_tuning(key, prev)
        lib().rt_set_variant(-1)


def test_trace_rays_matches_brute_force_closest_hit():
    """rt_trace_rays (v3's traversal without shading, tools/coherence.py) returns each ray's closest hit: against a
    numpy brute force over RTIOW's 488 spheres with Sphere::Hit's binary32 operations (Hittable.cuh:80-110: near
    root, else far root, strictly inside (0.001, FLT_MAX)), the hit distances are equal bit for bit, in any ray order."""
    sc = scenes.builtin(scenes.CONFIGS["c2"].scene)
    ds = DeviceScene(sc)
    rng = np.random.default_rng(5)
    n = 8192
    o = np.stack([rng.uniform(-12, 12, n), rng.uniform(0.05, 3.0, n), rng.uniform(-12, 12, n)], 1).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d[: n // 4, 1] = -np.abs(d[: n // 4, 1])  # a quarter aimed down at the small spheres and the ground
    rays = np.zeros((2 * n, 4), np.float32)
    rays[0::2, :3], rays[1::2, :3] = o, d
    # brute force (float32 throughout, the kernel's operation order)
    c = np.array([list(h.center) for h in sc.hittables], np.float32)
    r2 = np.array([h.radius * h.radius for h in sc.hittables], np.float32)
    f = np.float32
    best = np.full(n, np.inf, np.float32)
    a = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
    for k in range(len(c)):
        oc = o - c[k]
        b = (oc[:, 0] * d[:, 0] + oc[:, 1] * d[:, 1]) + oc[:, 2] * d[:, 2]
        cc = ((oc[:, 0] * oc[:, 0] + oc[:, 1] * oc[:, 1]) + oc[:, 2] * oc[:, 2]) - r2[k]
        disc = b * b - a * cc
        with np.errstate(invalid="ignore"):
            sq = np.sqrt(np.where(disc > 0, disc, f(1.0)))
            tn, tf = (-b - sq) / a, (-b + sq) / a
        t = np.where(tn > f(0.001), tn, np.where(tf > f(0.001), tf, np.inf)).astype(np.float32)
        t = np.where(disc > 0, t, np.inf)
        best = np.minimum(best, t)
    for perm in (np.arange(n), rng.permutation(n)):
        dr = torch.from_numpy(np.ascontiguousarray(rays.reshape(n, 8)[perm].reshape(2 * n, 4))).cuda()
        hits = torch.empty(2 * n, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(abi.COUNTERS_WORDS, dtype=torch.int64, device="cuda")
        assert lib().rt_trace_rays(ds.handle, C.c_void_p(dr.data_ptr()), n, C.c_void_p(hits.data_ptr()),
                                   C.c_void_p(cnt.data_ptr()), 1, None) == 0
        torch.cuda.synchronize()
        h = hits.cpu().numpy().reshape(n, 2)
        got = np.where(h[:, 0] >= 0, h[:, 1].view(np.float32), np.inf)
        want = best[perm]
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
        assert int(cnt[0]) == n and int(cnt[1]) > 2 * n
    assert np.isfinite(best).mean() > 0.3



# (RT_TUNE_PERSISTENT_GROUP, RT_TUNE_GROUP_TAIL, RT_TUNE_GROUP_ORDER, RT_TUNE_QUEUE_RESET)
GROUP_KNOBS = [(1, 0, 0, 0), (1, 0, 1, 0), (1, 100, 0, 0), (1, 1000, 0, 0), (1, 300, 1, 1), (0, 0, 0, 0), (0, 0, 0, 1),
               (2, 0, 0, 0), (2, 0, 0, 1)]


@pytest.mark.parametrize("group, tail, order, reset", GROUP_KNOBS, ids=lambda v: str(v))
def test_persistent_flat_group_knobs_change_schedule_not_pixels(group, tail, order, reset):
    """The persistent flat kernel's workgroup shares (round 6): 16-wave groups handing a static share of the tiles to
    their lanes through an LDS counter, the per-wave queue behind them (RT_TUNE_GROUP_TAIL permille of the tiles), the
    shares' order, and the queue slot's reset (in-kernel by the last group or wave, or a host memset) decide which lane
    renders which pixel, never what it computes: every setting gives the golden image, ray count and RNG states, on a
    textured scene (C5's) and on the Cornell box, frame after frame on the reused queue slots."""
    keys = (abi.RT_TUNE_PERSISTENT_GROUP, abi.RT_TUNE_GROUP_TAIL, abi.RT_TUNE_GROUP_ORDER, abi.RT_TUNE_QUEUE_RESET)
    prev = [lib().rt_set_tuning(k, v) for k, v in zip(keys, (group, tail, order, reset))]
    assert min(prev) >= 0
    lib().rt_set_variant(6)
    try:
        for name in ("c5_textured_160x96_s4", "c3_cornell_128_s16"):
            case = CASE_BY_NAME[name]
            cfg, g = case.cfg(), load_golden(case.name)
            ds = DeviceScene(scenes.builtin(cfg.scene))
            for _ in range(2):
                r = Renderer(cfg.width, cfg.height)
                r.render_init()
                r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=case.flags)
                torch.cuda.synchronize()
                assert lib().rt_last_variant() == 6
                np.testing.assert_array_equal(r.image(), g["pos"], err_msg=name)
                assert digest(r.states()[:, :6]) == g["state_after_sha256"].tobytes(), name
                assert int(r.counters[0]) == int(g["counters"][0]), name
    finally:
        lib().rt_set_variant(-1)
        for k, v in zip(keys, prev):
            lib().rt_set_tuning(k, v)


@pytest.mark.parametrize("chunk", [64, 128, 1024, 4096])
def test_persistent_flat_group_queue_chunks(chunk):
    """The workgroup chunk queue (RT_TUNE_PERSISTENT_GROUP 2): any chunk size — from one tile per chunk to chunks
    larger than a small frame's share of a queue head — renders the golden image, rays and RNG states."""
    keys = (abi.RT_TUNE_PERSISTENT_GROUP, abi.RT_TUNE_GROUP_CHUNK)
    prev = [lib().rt_set_tuning(k, v) for k, v in zip(keys, (2, chunk))]
    assert min(prev) >= 0
    lib().rt_set_variant(6)
    try:
        for name in ("c5_textured_160x96_s4", "c3_cornell_128_s16"):
            case = CASE_BY_NAME[name]
            cfg, g = case.cfg(), load_golden(case.name)
            r = Renderer(cfg.width, cfg.height)
            r.render_init()
            r.render(DeviceScene(scenes.builtin(cfg.scene)), cfg.spp, cfg.depth, cfg.inputs(), flags=case.flags)
            torch.cuda.synchronize()
            assert lib().rt_last_variant() == 6
            np.testing.assert_array_equal(r.image(), g["pos"], err_msg=name)
            assert digest(r.states()[:, :6]) == g["state_after_sha256"].tobytes(), name
            assert int(r.counters[0]) == int(g["counters"][0]), name
    finally:
        lib().rt_set_variant(-1)
        for k, v in zip(keys, prev):
            lib().rt_set_tuning(k, v)


@pytest.mark.parametrize("waves, group", [(4, 2), (8, 2), (12, 2), (12, 1)])
def test_persistent_flat_group_sizes(waves, group):
    """Workgroups of 4, 8 or 12 waves instead of 16 (RT_TUNE_GROUP_WAVES), with the chunk queue and with static shares:
    the golden image, rays and RNG states."""
    keys = (abi.RT_TUNE_PERSISTENT_GROUP, abi.RT_TUNE_GROUP_WAVES)
    prev = [lib().rt_set_tuning(k, v) for k, v in zip(keys, (group, waves))]
    assert min(prev) >= 0
    lib().rt_set_variant(6)
    try:
        for name in ("c5_textured_160x96_s4", "c3_cornell_128_s16"):
            case = CASE_BY_NAME[name]
            cfg, g = case.cfg(), load_golden(case.name)
            r = Renderer(cfg.width, cfg.height)
            r.render_init()
            r.render(DeviceScene(scenes.builtin(cfg.scene)), cfg.spp, cfg.depth, cfg.inputs(), flags=case.flags)
            torch.cuda.synchronize()
            assert lib().rt_last_variant() == 6
            np.testing.assert_array_equal(r.image(), g["pos"], err_msg=name)
            assert digest(r.states()[:, :6]) == g["state_after_sha256"].tobytes(), name
            assert int(r.counters[0]) == int(g["counters"][0]), name
    finally:
        lib().rt_set_variant(-1)
        for k, v in zip(keys, prev):
            lib().rt_set_tuning(k, v)
