"""CPU tests of librt_hip.so's host code: scene generators, glibc rand restatement, camera set-up, scene
validation, the BVH build and the reference-graph flattener (no device needed)."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import pytest

import refgraph
from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd._lib import lib
from helpers import load_golden


def test_glibc_rand_restatement_matches_libc():
    libc = C.CDLL("libc.so.6")
    for seed in (1, 42, 1984):
        g = abi.GlibcRand()
        lib().rt_glibc_srand(C.byref(g), seed)
        libc.srand(seed)
        assert [lib().rt_glibc_rand_next(C.byref(g)) for _ in range(3000)] == [libc.rand() for _ in range(3000)]


@pytest.mark.parametrize("which", range(5))
def test_builtin_scenes_match_golden(which):
    s = scenes.builtin(which)
    g = load_golden(f"scene_{which}")
    assert s.hittables_bytes() == g["hittables"].tobytes()
    assert s.materials_bytes() == g["materials"].tobytes()


def test_builtin_scene_shapes():
    rtiow = scenes.builtin(scenes.SCENE_RTIOW)
    assert rtiow.num_hittables == 488  # 1 ground + 22×22 + 3
    kinds = [rtiow.materials[h.material].type for h in rtiow.hittables]
    assert kinds.count(abi.RT_DIELECTRIC) >= 1 and kinds.count(abi.RT_METAL) >= 1
    world = scenes.builtin(scenes.SCENE_DEFAULT_WORLD)
    assert world.num_hittables == 17 and world.hittables[0].type == abi.RT_XZRECT
    assert world.materials[0].albedo.type == abi.RT_CHECKER
    for h in list(world.hittables)[1:]:
        m = world.materials[h.material]
        assert h.type == abi.RT_SPHERE
        assert h.radius == pytest.approx({abi.RT_LAMBERTIAN: 0.2, abi.RT_METAL: 0.2, abi.RT_DIELECTRIC: 0.3,
                                          abi.RT_DIFFUSELIGHT: 0.5}[m.type])
        if m.type == abi.RT_METAL:
            assert 0 <= m.fuzz <= 0.5
    cornell = scenes.builtin(scenes.SCENE_CORNELL)
    assert {h.type for h in cornell.hittables} == {abi.RT_XYRECT, abi.RT_XZRECT, abi.RT_YZRECT, abi.RT_SPHERE}


def test_camera_inputs_reference_up_vector():
    """CudaLayer.cpp:45-46 passes up = normalize(cross(o, normalize(cross(o, worldUp)))): down for a level camera."""
    inp = scenes.camera_inputs((0.0, 2.0, 12.0), (0.0, 0.0, -1.0), 45.0)
    assert list(inp.up) == [0.0, -1.0, 0.0]
    assert inp.fov == pytest.approx(np.radians(45.0), rel=1e-7)
    assert (inp.near_plane, inp.far_plane) == (pytest.approx(0.1), 10.0)
    assert list(inp.background_start) == [1.0, 1.0, 1.0] and list(inp.background_end) == pytest.approx([0.5, 0.7, 1.0])
    assert C.sizeof(inp) == 72


def _tables(scene):
    desc = scene.desc()
    info = abi.HostTablesInfo()
    assert lib().rt_build_host_tables(C.byref(desc), None, None, None, None, C.byref(info)) == 0
    nodes = (C.c_float * (16 * info.num_nodes))()
    prims = (C.c_float * (8 * info.num_prims))()
    mats = (C.c_float * (12 * info.num_materials))()
    src = (C.c_int32 * max(1, info.num_prims))()
    assert lib().rt_build_host_tables(C.byref(desc), nodes, prims, mats, src, C.byref(info)) == 0
    return (info, np.frombuffer(nodes, np.float32).reshape(-1, 16), np.frombuffer(prims, np.float32).reshape(-1, 8),
            np.frombuffer(src, np.int32)[: info.num_prims])


@pytest.mark.parametrize("which", range(5))
def test_bvh_covers_every_active_primitive_once_with_conservative_boxes(which):
    scene = scenes.builtin(which)
    info, nodes, prims, src = _tables(scene)
    active = [i for i in range(scene.num_hittables) if scene.hittables[i].is_active]
    assert sorted(src.tolist()) == active
    ints = nodes.view(np.int32)
    seen = []

    def prim_box(i):
        h = scene.hittables[int(src[i])]
        c = np.float32(h.center)
        if h.type == abi.RT_SPHERE:
            return c - np.float32(h.radius), c + np.float32(h.radius)
        k = {abi.RT_XYRECT: 2, abi.RT_XZRECT: 1, abi.RT_YZRECT: 0}[h.type]
        lo, hi = prims[i, [1, 3]], prims[i, [2, 4]]
        axes = {2: (0, 1), 1: (0, 2), 0: (1, 2)}[k]
        blo, bhi = np.zeros(3, np.float32), np.zeros(3, np.float32)
        blo[list(axes)], bhi[list(axes)] = lo, hi
        blo[k], bhi[k] = c[k] - np.float32(1e-4), c[k] + np.float32(1e-4)
        return blo, bhi

    def walk(child, lo, hi, depth):
        assert depth <= info.depth
        if child < 0:
            leaf = ~child
            first, count = leaf >> 2, (leaf & 3) + 1
            assert 1 <= count <= 4
            for i in range(first, first + count):
                seen.append(i)
                plo, phi = prim_box(i)
                assert np.all(lo < plo) and np.all(hi > phi), (lo, hi, plo, phi)  # strictly padded outward
            return
        n = nodes[child]
        boxes = [(n[[0, 2, 8]], n[[1, 3, 9]]), (n[[4, 6, 10]], n[[5, 7, 11]])]
        for k in range(2):
            blo, bhi = boxes[k]
            assert np.all(blo >= lo) and np.all(bhi <= hi)
            walk(int(ints[child, 12 + k]), blo, bhi, depth + 1)

    inf = np.float32(np.inf)
    walk(0, np.full(3, -inf), np.full(3, inf), 1)
    if info.num_prims == 1:
        assert seen == [0, 0]
    else:
        assert sorted(seen) == list(range(info.num_prims))


def test_bvh_is_shallow_and_small_for_rtiow():
    info, nodes, _, _ = _tables(scenes.builtin(scenes.SCENE_RTIOW))
    assert info.num_prims == 488 and info.depth <= 24
    assert nodes.nbytes + info.num_prims * 32 <= 48 * 1024  # LDS-stageable


def test_bvh_depth_guard_keeps_eight_wave_occupancy():
    """A cheap node-visit SAH cost makes RTIOW's tree 13 levels deep, one more than the compact v3 kernel's LDS
    holds at 8 waves/SIMD: the builder retries with dearer visits until the tree fits (scene_build.cpp)."""
    prev = lib().rt_set_tuning(3, 6)
    try:
        info, nodes, _, _ = _tables(scenes.builtin(scenes.SCENE_RTIOW))
        assert info.depth <= 12 and info.num_prims == 488
    finally:
        lib().rt_set_tuning(3, prev)
    info, _, _, _ = _tables(scenes.builtin(scenes.SCENE_RTIOW))  # the default tree fits as built
    assert info.depth <= 12


def test_inactive_hittables_are_dropped():
    s = scenes.builtin(scenes.SCENE_DEFAULT_WORLD)
    s.hittables[3].is_active = 0
    s.hittables[7].is_active = 0
    _, _, _, src = _tables(s)
    assert 3 not in src.tolist() and 7 not in src.tolist() and len(src) == 15


def test_empty_and_single_primitive_scenes():
    s = scenes.builtin(scenes.SCENE_THREE_SPHERES)
    for h in s.hittables:
        h.is_active = 0
    info, _, _, _ = _tables(s)
    assert info.num_nodes == 0 and info.num_prims == 0
    s.hittables[1].is_active = 1
    info, nodes, _, src = _tables(s)
    assert info.num_nodes == 1 and src.tolist() == [1]


@pytest.mark.parametrize("mutate, code", [
    (lambda s: setattr(s.hittables[0], "material", 99), -2),
    (lambda s: setattr(s.hittables[0], "type", 7), -2),
    (lambda s: setattr(s.materials[0], "type", 9), -2),
    (lambda s: setattr(s.materials[0].albedo, "type", 5), -2),
    (lambda s: s.hittables[1].center.__setitem__(2, float("nan")), -2),  # no box for NaN geometry
    (lambda s: setattr(s.hittables[0], "radius", float("inf")), -2),
    (lambda s: setattr(s.hittables[0], "radius", -0.5), -2),  # inside-out reference box (Hittable.cuh:114)
])
def test_invalid_scenes_are_rejected(mutate, code):
    s = scenes.builtin(scenes.SCENE_THREE_SPHERES)
    mutate(s)
    desc = s.desc()
    info = abi.HostTablesInfo()
    assert lib().rt_build_host_tables(C.byref(desc), None, None, None, None, C.byref(info)) == code
    assert lib().rt_last_error()
    handle = C.c_void_p()
    assert lib().rt_scene_create(C.byref(desc), C.byref(handle)) == code  # validation precedes any device call


@pytest.mark.parametrize("which", [scenes.SCENE_DEFAULT_WORLD, scenes.SCENE_CORNELL, scenes.SCENE_TEXTURED])
def test_reference_graph_flattens_to_the_same_scene(which):
    s = scenes.builtin(which)
    g = refgraph.build_graph(s)
    nh, nm, ni = C.c_uint32(0), C.c_uint32(0), C.c_uint32(0)
    world = C.addressof(g.world)
    assert lib().rt_reference_graph_flatten(world, None, C.byref(nh), None, C.byref(nm), None, C.byref(ni)) == 0
    h = (abi.HittableDesc * nh.value)()
    m = (abi.MaterialDesc * nm.value)()
    im = (abi.ImageDesc * max(1, ni.value))()
    assert lib().rt_reference_graph_flatten(world, h, C.byref(nh), m, C.byref(nm), im, C.byref(ni)) == 0
    assert nh.value == s.num_hittables
    # same primitives and materials (order may differ: the graph is walked in BVH order)
    want = sorted((bytes(x.center), x.type, x.radius, x.width, x.height, bytes(s.materials[x.material]))
                  for x in s.hittables)
    got = []
    for x in h:
        mm = m[x.material]
        if mm.albedo.type == abi.RT_IMAGE:  # one image per textured material in the graph: map it back
            mm.albedo.image = [np.asarray(i).ctypes.data for i in s.images].index(im[mm.albedo.image].data)
        got.append((bytes(x.center), x.type, x.radius, x.width, x.height, bytes(mm)))
    assert sorted(got) == want


def test_reference_graph_rejects_non_bvh_world():
    bad = refgraph.Hittable()
    bad.type = abi.RT_SPHERE
    nh, nm, ni = C.c_uint32(0), C.c_uint32(0), C.c_uint32(0)
    assert lib().rt_reference_graph_flatten(C.addressof(bad), None, C.byref(nh), None, C.byref(nm), None,
                                            C.byref(ni)) == -2


def test_scheduling_knobs_defaults_and_ranges():
    """rt_set_tuning for the v3 scheduling knobs (CPU: no kernel runs): round-3 defaults, range checks, and the
    previous value returned (include/rt_hip.h rt_tuning_key)."""
    L = lib()
    for key, default, bad in [(abi.RT_TUNE_REGEN_THRESHOLD, 56, [0, 65]), (abi.RT_TUNE_REGEN_LIVE_FRAC, 48, [-1, 65]),
                              (abi.RT_TUNE_LEAF_BREAK, 3, [-1, 65]), (abi.RT_TUNE_RIUS_TRIPS, 4, [-1, 65]),
                              (abi.RT_TUNE_RIUS_TRIPS_PERSISTENT, 0, [-1, 65])]:
        prev = L.rt_set_tuning(key, 7)
        assert prev == default, (key, prev)
        assert L.rt_set_tuning(key, prev) == 7
        for b in bad:
            assert abi.STATUS.get(L.rt_set_tuning(key, b)) == "RT_ERR_INVALID_ARGUMENT", (key, b)
        assert L.rt_set_tuning(key, default) == default  # unchanged by the refused values


def test_queue_knobs_defaults_and_ranges():
    """rt_set_tuning for the persistent kernels' queue (CPU: no kernel runs): chunk (multiple of 64), head stride
    (power of two), chunk prefetch threshold (include/rt_hip.h RT_TUNE_QUEUE_PREFETCH)."""
    L = lib()
    for key, default, good, bad in [(abi.RT_TUNE_QUEUE_CHUNK, 128, 192, [0, 96, 4160]),
                                    (abi.RT_TUNE_QUEUE_STRIDE, 128, 4096, [64, 192, 8192]),
                                    (abi.RT_TUNE_QUEUE_PREFETCH, QUEUE_PREFETCH_DEFAULT, 48, [-1, 65]),
                                    (abi.RT_TUNE_QUEUE_GUIDE, QUEUE_GUIDE_DEFAULT, 4, [-1, 65]),
                                    (abi.RT_TUNE_QUEUE_MIN_CHUNK, 16, 32, [0, 24, 80])]:
        prev = L.rt_set_tuning(key, good)
        assert prev == default, (key, prev)
        for b in bad:
            assert abi.STATUS.get(L.rt_set_tuning(key, b)) == "RT_ERR_INVALID_ARGUMENT", (key, b)
        assert L.rt_set_tuning(key, default) == good


QUEUE_PREFETCH_DEFAULT = 32
QUEUE_GUIDE_DEFAULT = 0


# ---------------------------------------------------------------------------------------------------
# Image loading (LoadImage, Utils/RawStbImage.h:11-22) and the reference's own texture assets
# ---------------------------------------------------------------------------------------------------
REF_TEXTURES = "/root/reference/assets/textures"


def test_load_image_mirrors_loadimage(tmp_path):
    from PIL import Image

    rgb = (np.arange(5 * 7 * 3, dtype=np.uint8) * 7).reshape(5, 7, 3)
    Image.fromarray(rgb).save(tmp_path / "a.png")
    got = scenes.load_image(str(tmp_path / "a.png"))
    assert got.shape == (5, 7, 3) and np.array_equal(got, rgb)  # row 0 at the top, as stb decodes
    grey = rgb[:, :, 0]
    Image.fromarray(grey).save(tmp_path / "g.png")
    assert scenes.load_image(str(tmp_path / "g.png")).shape == (5, 7, 1)  # channels as stored (desired_channels 0)
    assert scenes.load_image(str(tmp_path / "missing.jpg")) is None  # the reference logs and returns nullptr
    (tmp_path / "bad.jpg").write_bytes(b"not a jpeg")
    assert scenes.load_image(str(tmp_path / "bad.jpg")) is None


def test_textured_scene_takes_caller_images():
    imgs = [np.full((64, 128, 3), v, dtype=np.uint8) for v in (10, 20, 30)]
    sc = scenes.builtin(scenes.SCENE_TEXTURED, images=imgs)
    assert [im.shape for im in sc.images] == [(64, 128, 3)] * 3
    with pytest.raises(ValueError):
        scenes.builtin(scenes.SCENE_TEXTURED, images=imgs[:2])
    with pytest.raises(ValueError):
        scenes.builtin(scenes.SCENE_TEXTURED, images=[imgs[0], imgs[1], imgs[2][:, :, :1]])


@pytest.mark.skipif(not os.path.isdir(REF_TEXTURES), reason="the reference's assets are not here")
def test_reference_texture_files_load_as_rgb8():
    """The reference's own planet maps, read in place (nothing derived from them is stored): each decodes to the
    RGB8 layout Image::value reads (Texture.cuh:76) and sits on the textured scene's spheres."""
    imgs = [scenes.load_image(os.path.join(REF_TEXTURES, n)) for n in ("8k_earth_nightmap.jpg", "8k_stars.jpg",
                                                                        "8k_sun.jpg")]
    assert [im.shape for im in imgs] == [(4096, 8192, 3), (4096, 8192, 3), (2048, 4096, 3)]
    sc = scenes.builtin(scenes.SCENE_TEXTURED, images=imgs)
    d = sc.desc()
    assert d.num_images == 3 and (d.images[2].width, d.images[2].height) == (4096, 2048)
