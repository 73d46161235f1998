"""CPU tests of the oracle (oracle/rt_oracle.c): pinned against the survey-recorded reference values and the
committed golden fixtures, plus analytical known-answer tests of each restated function."""
from __future__ import annotations

import ctypes as C
import json
import math
import os
import struct

import numpy as np
import pytest

from cases import CASE_BY_NAME, CASES, PHILOX_CASES
from cudaraytracer_amd import abi, scenes
from helpers import GOLDEN, digest, load_golden
from oracle import py_oracle as po

pytestmark = pytest.mark.filterwarnings("ignore")


# ---------------------------------------------------------------------------------------------------
# Pins from SURVEY.md §8(c) C1 / §6 (outputs of the reference's own hot-path source, survey probe)
# ---------------------------------------------------------------------------------------------------
def test_xorwow_kat_matches_survey_probe():
    st = abi.CurandState()
    po.lib().orc_curand_init(1984, C.byref(st))
    got = [po.lib().orc_curand_uniform(C.byref(st)) for _ in range(3)]
    assert got == pytest.approx([0.195986241, 0.454007715, 0.358994216], abs=5e-10)


def test_c1_matches_survey_probe():
    """BASELINE config 1 through the reference grid: px(200,112)=0xff7f5f3c, px(0,0)=0xff00c0a4, row 224
    unwritten, 868,442 rays, 4.0 box tests/ray."""
    cfg = scenes.CONFIGS["c1"]
    sc = scenes.builtin(cfg.scene)
    st = po.init_states(cfg.width, cfg.height, full=False)
    pos, _, cnt = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st,
                            faithful_grid=True, rius_order=1)
    assert pos[112, 200] == 0xFF7F5F3C
    assert pos[0, 0] == 0xFF00C0A4
    assert not pos[224].any() and pos[224, 399] == 0
    assert cnt.rays == 868442
    assert cnt.box_tests / cnt.rays == pytest.approx(4.0, abs=0.01)
    # the survey's checksum (definition not recorded) is 26,494,510; Σ RGB here is within 1 of it
    s = int(pos.view(np.uint8).reshape(-1, 4)[:, :3].sum())
    assert abs(s - 26494510) <= 1


def test_c1_left_to_right_order_differs_from_probe():
    """The probe's g++ build filled Random()'s Vec3 right to left; left to right gives another image."""
    cfg = scenes.CONFIGS["c1"]
    sc = scenes.builtin(cfg.scene)
    st = po.init_states(cfg.width, cfg.height, full=False)
    pos, _, cnt = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st,
                            faithful_grid=True, rius_order=0)
    assert pos[112, 200] != 0xFF7F5F3C and cnt.rays != 868442


def test_xorwow_recurrence_matches_rocrand_engine():
    """tests/golden/rocrand_xorwow_kat.json is rocRAND's own xorwow engine (make_rocrand_xorwow_kat.cpp): the
    oracle's seeding with rocRAND's four constants must give rocRAND's state, and orc_curand (cuRAND's
    curand(), the recurrence both libraries share) its outputs.  cuRAND's own four seeding constants are
    pinned by the survey probe above."""
    with open(os.path.join(GOLDEN, "rocrand_xorwow_kat.json")) as f:
        kat = json.load(f)
    k = kat["seeding_constants"]
    assert len(kat["streams"]) >= 8
    for v in kat["streams"]:
        st = abi.CurandState()
        po.lib().orc_xorwow_seed(v["seed"], k["xor0"], k["xor1"], k["mul0"], k["mul1"], C.byref(st))
        assert [st.d] + list(st.v) == v["init"], v["seed"]
        assert [po.lib().orc_curand(C.byref(st)) for _ in range(len(v["raw"]))] == v["raw"], v["seed"]


# ---------------------------------------------------------------------------------------------------
# Golden fixtures (regression of the restatement; tests/golden/make_golden.py)
# ---------------------------------------------------------------------------------------------------
def test_xorwow_golden():
    with open(os.path.join(GOLDEN, "xorwow_kat.json")) as f:
        kat = json.load(f)
    for seed, v in kat.items():
        st = abi.CurandState()
        po.lib().orc_curand_init(int(seed), C.byref(st))
        assert [st.d] + list(st.v) == v["init"]
        assert [po.lib().orc_curand(C.byref(st)) for _ in range(8)] == v["raw"]


@pytest.mark.parametrize("case", CASES, ids=lambda c: c.name)
def test_oracle_matches_golden(case):
    g = load_golden(case.name)
    cfg = case.cfg()
    sc = scenes.builtin(cfg.scene)
    inp = abi.InputStruct.from_buffer_copy(g["inputs"].tobytes())
    assert bytes(inp) == bytes(cfg.inputs())
    st = po.init_states(cfg.width, cfg.height, full=not case.faithful_grid)
    assert digest(st[:, :6]) == g["state_before_sha256"].tobytes()
    pos, rad, cnt = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, inp, st,
                              faithful_grid=case.faithful_grid, rius_order=case.rius_order, radiance=True)
    np.testing.assert_array_equal(pos, g["pos"])
    assert digest(st[:, :6]) == g["state_after_sha256"].tobytes()
    assert digest(rad) == g["radiance_sha256"].tobytes()
    assert [cnt.rays, cnt.box_tests, cnt.prim_tests, cnt.primary] == [int(x) for x in g["counters"]]


@pytest.mark.parametrize("case", [c for c in CASES if c.spp <= 8 or c.width <= 128], ids=lambda c: c.name)
def test_reference_bvh_culling_equals_exact_closest_hit(case):
    """The reference BVH + AABB culling returns the geometric closest hit on every golden case."""
    cfg = case.cfg()
    sc = scenes.builtin(cfg.scene)
    out = []
    for exact in (False, True):
        st = po.init_states(cfg.width, cfg.height)
        pos, _, cnt = po.render(po.OracleScene(sc, exact=exact), cfg.width, cfg.height, cfg.spp, cfg.depth,
                                cfg.inputs(), st, rius_order=case.rius_order)
        out.append((pos, cnt.rays))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]


def test_row_sampling_matches_full_frame():
    cfg = scenes.CONFIGS["c2"].scaled(64, 40, 2)
    sc = po.OracleScene(scenes.builtin(cfg.scene))
    st_full = po.init_states(cfg.width, cfg.height)
    full, _, _ = po.render(sc, cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st_full)
    st = po.init_states(cfg.width, cfg.height)
    part, _, cnt = po.render(sc, cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st, rows=(3, 40), row_step=5)
    rows = list(range(3, 40, 5))
    np.testing.assert_array_equal(part[rows], full[rows])
    assert cnt.primary == len(rows) * cfg.width * cfg.spp


# ---------------------------------------------------------------------------------------------------
# Known-answer tests of the restated functions
# ---------------------------------------------------------------------------------------------------
def _hit(h, o, d, tmin=0.001, tmax=3.4e38):
    out = po.Hit()
    F3 = C.c_float * 3
    po.lib().orc_hittable_hit(C.byref(h), F3(*o), F3(*d), tmin, tmax, C.byref(out))
    return out


def _sphere(c, r):
    h = abi.HittableDesc()
    h.type, h.is_active, h.radius = abi.RT_SPHERE, 1, r
    h.center[:] = c
    return h


def _rect(t, c, w, hh):
    h = abi.HittableDesc()
    h.type, h.is_active, h.width, h.height = t, 1, w, hh
    h.center[:] = c
    return h


def test_sphere_hit_near_and_far_root():
    s = _sphere((0.0, 0.0, -5.0), 1.0)
    h = _hit(s, (0, 0, 0), (0, 0, -1))
    assert h.hit and h.t == pytest.approx(4.0) and list(h.normal) == pytest.approx([0, 0, 1])
    # GetSphereUV of the normal (0,0,1): u = (atan2(-1, 0) + π)/2π = 0.25, v = acos(0)/π = 0.5
    assert h.u == pytest.approx(0.25, abs=1e-6) and h.v == pytest.approx(0.5, abs=1e-6)
    inside = _hit(s, (0, 0, -5), (0, 0, -1))  # origin inside: near root < tmin → far root
    assert inside.hit and inside.t == pytest.approx(1.0)
    assert list(inside.normal) == pytest.approx([0, 0, -1])  # outward, NOT face-flipped (Hittable.cuh:93)
    assert not _hit(s, (0, 0, 0), (0, 1, 0)).hit
    assert not _hit(s, (0, 0, 0), (0, 0, -1), tmax=4.0).hit  # strict t < t_max
    assert not _hit(s, (0, 0, 0), (0, 0, -1), tmin=6.0).hit  # both roots <= t_min


def test_rect_hits_and_face_normals():
    xy = _rect(abi.RT_XYRECT, (0.0, 0.0, -2.0), 2.0, 4.0)
    h = _hit(xy, (0.5, 1.0, 0.0), (0, 0, -1))
    assert h.hit and h.t == pytest.approx(2.0)
    assert (h.u, h.v) == pytest.approx((0.75, 0.75))
    assert list(h.normal) == pytest.approx([0, 0, 1]) and h.front_face == 1
    back = _hit(xy, (0.5, 1.0, -4.0), (0, 0, 1))
    assert back.hit and list(back.normal) == pytest.approx([0, 0, -1]) and back.front_face == 0
    assert not _hit(xy, (1.5, 0.0, 0.0), (0, 0, -1)).hit  # outside x extent
    xz = _rect(abi.RT_XZRECT, (0.0, -0.5, 0.0), 1000.0, 1000.0)
    g = _hit(xz, (0.0, 2.0, 12.0), (0.0, -1.0, 0.0))
    assert g.hit and g.t == pytest.approx(2.5) and list(g.normal) == pytest.approx([0, 1, 0])
    # YZ: width spans z, height spans y (Hittable.cuh:255-258)
    yz = _rect(abi.RT_YZRECT, (3.0, 0.0, 0.0), 10.0, 2.0)
    assert _hit(yz, (0.0, 0.0, 4.0), (1, 0, 0)).hit
    assert not _hit(yz, (0.0, 4.0, 0.0), (1, 0, 0)).hit
    # rect acceptance is inclusive in t (t > t_max rejects, t == t_max accepts)
    assert _hit(xy, (0.0, 0.0, 0.0), (0, 0, -1), tmax=2.0).hit


def _scatter(mat, o, d, hit, seed=1984, order=1):
    st = abi.CurandState()
    po.lib().orc_curand_init(seed, C.byref(st))
    F3 = C.c_float * 3
    so, sd, att = F3(), F3(), F3()
    draws = C.c_int(0)
    ok = po.lib().orc_scatter(C.byref(mat), F3(*o), F3(*d), C.byref(hit), C.byref(st), so, sd, att,
                              C.byref(draws), order)
    return ok, list(so), list(sd), list(att), draws.value, st


def _mat(t, color=(0.5, 0.5, 0.5), fuzz=0.0, ir=1.5):
    m = abi.MaterialDesc()
    m.type, m.fuzz, m.ir = t, fuzz, ir
    m.albedo.type = abi.RT_CONSTANT
    m.albedo.color[:] = color
    return m


def _uniforms(seed, n):
    st = abi.CurandState()
    po.lib().orc_curand_init(seed, C.byref(st))
    return [po.lib().orc_curand_uniform(C.byref(st)) for _ in range(n)]


def test_lambertian_scatter_direction_and_draws():
    hit = po.Hit(1, 2.0, (C.c_float * 3)(0.25, -0.5, 1.0), (C.c_float * 3)(0.0, 1.0, 0.0), 0.0, 0.0, 1)
    ok, so, sd, att, draws, _ = _scatter(_mat(abi.RT_LAMBERTIAN, (0.1, 0.2, 0.3)), (0, 1, 0), (0, -1, 0), hit)
    assert ok == 1 and att == pytest.approx([0.1, 0.2, 0.3]) and draws % 3 == 0 and draws >= 3
    # reproduce RandomInUnitSphere's accepted sample (right-to-left fill) and ((p + n) + q) - p
    u = _uniforms(1984, draws)
    a, b, c = u[-3:]
    q = [np.float32(2.0) * np.float32(c) - np.float32(1.0), np.float32(2.0) * np.float32(b) - np.float32(1.0),
         np.float32(2.0) * np.float32(a) - np.float32(1.0)]
    p, n = np.float32([0.25, -0.5, 1.0]), np.float32([0.0, 1.0, 0.0])
    want = ((p + n) + np.float32(q)) - p
    assert sd == [float(x) for x in want]
    assert so == [0.25, -0.5, 1.0]


def test_metal_scatter_absorbs_below_surface_and_always_draws():
    hit = po.Hit(1, 1.0, (C.c_float * 3)(0, 0, 0), (C.c_float * 3)(0, 1, 0), 0, 0, 1)
    ok, _, sd, att, draws, _ = _scatter(_mat(abi.RT_METAL, (0.9, 0.8, 0.7), fuzz=0.0), (0, 1, 0), (1, -1, 0), hit)
    assert ok == 1 and draws >= 3  # RNG drawn even with fuzz 0 (Material.cuh:79)
    assert sd == pytest.approx([1 / math.sqrt(2), 1 / math.sqrt(2), 0], abs=1e-6)
    ok2, _, sd2, _, _, _ = _scatter(_mat(abi.RT_METAL, fuzz=1.0), (0, 1, 0), (1, -1e-4, 0), hit, seed=7)
    assert ok2 == (1 if sd2[1] > 0 else 0)


def test_dielectric_total_internal_reflection_and_one_draw():
    # exiting ray at a grazing angle: sin θ_t = 1.5·sin θ_i > 1 → reflect with probability 1
    hit = po.Hit(1, 1.0, (C.c_float * 3)(0, 0, 0), (C.c_float * 3)(0, 1, 0), 0, 0, 1)
    ok, _, sd, att, draws, _ = _scatter(_mat(abi.RT_DIELECTRIC), (0, -1, 0), (1.0, 0.2, 0.0), hit)
    assert ok == 1 and att == [1.0, 1.0, 1.0] and draws == 1
    assert sd == pytest.approx([1.0, -0.2, 0.0])  # un-normalized Reflect(d, n)
    # normal incidence from outside: Schlick r0 = 0.04 → refract unless ξ < 0.04
    ok, _, sd, _, draws, _ = _scatter(_mat(abi.RT_DIELECTRIC), (0, 1, 0), (0.0, -1.0, 0.0), hit)
    xi = _uniforms(1984, 1)[0]
    assert draws == 1
    assert sd == pytest.approx([0.0, 1.0, 0.0] if xi < 0.04 else [0.0, -1.0, 0.0])


def test_rgb_to_int_clamps_truncates_and_nan():
    f = po.lib().orc_rgb_to_int
    assert f(0.0, 0.0, 0.0) == 0xFF000000
    assert f(255.9, 300.0, -5.0) == 0xFF00FFFF
    assert f(12.99, 1.5, 128.0) == 0xFF80010C
    assert f(float("nan"), 3.0, 0.0) == 0xFF000300


# ---------------------------------------------------------------------------------------------------
# Perf-mode RNG: Philox4x32-10 (RT_FLAG_RNG_PHILOX), pinned to rocRAND's own engine and Random123's KATs
# ---------------------------------------------------------------------------------------------------
def _bits(f: float) -> int:
    return struct.unpack("<I", struct.pack("<f", f))[0]


def test_philox_matches_rocrand_engine():
    """tests/golden/philox_kat.json was produced by rocRAND's philox4x32_10 (make_philox_kat.cpp)."""
    with open(os.path.join(GOLDEN, "philox_kat.json")) as f:
        kat = json.load(f)
    U4, U2 = C.c_uint * 4, C.c_uint * 2
    for st in kat["streams"]:
        seed, pixel, frame = st["seed"], st["pixel"], st["frame"]
        got = [_bits(po.lib().orc_philox_uniform_at(seed, pixel, frame, n)) for n in range(11)]
        assert got == st["uniform_bits"], st
        raw = []
        for blk in range(3):
            out = U4()
            po.lib().orc_philox4x32_10(U4(blk, frame, pixel & 0xFFFFFFFF, pixel >> 32),
                                       U2(seed & 0xFFFFFFFF, seed >> 32), out)
            raw += list(out)
        assert raw[:11] == st["raw"]


def test_philox_random123_known_answers():
    """Published Random123 known-answer vectors for philox4x32_10."""
    U4, U2 = C.c_uint * 4, C.c_uint * 2
    cases = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
             ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
             ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
              (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]
    for ctr, key, want in cases:
        out = U4()
        po.lib().orc_philox4x32_10(U4(*ctr), U2(*key), out)
        assert tuple(out) == want


@pytest.mark.parametrize("case, frame", PHILOX_CASES, ids=lambda x: getattr(x, "name", str(x)))
def test_oracle_philox_matches_golden(case, frame):
    g = load_golden(f"philox_{case.name}_f{frame}")
    cfg = case.cfg()
    pos, rad, cnt = po.render(po.OracleScene(scenes.builtin(cfg.scene)), cfg.width, cfg.height, cfg.spp, cfg.depth,
                              cfg.inputs(), None, faithful_grid=case.faithful_grid, rius_order=case.rius_order,
                              radiance=True, philox=True, seed=1984, frame=frame)
    np.testing.assert_array_equal(pos, g["pos"])
    assert digest(rad) == g["radiance_sha256"].tobytes()
    assert [cnt.rays, cnt.box_tests, cnt.prim_tests, cnt.primary] == [int(x) for x in g["counters"]]


def test_philox_mode_estimates_the_same_image():
    """Perf mode is a different random stream, not a different estimator: per channel, the mean over the
    image of (philox − xorwow) pre-gamma radiance is zero within 4 standard errors."""
    cfg = scenes.CONFIGS["c2"].scaled(128, 72, 16)
    sc = po.OracleScene(scenes.builtin(cfg.scene))
    st = po.init_states(cfg.width, cfg.height)
    _, rx, cx = po.render(sc, cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st, radiance=True, threads=8)
    _, rp, cp = po.render(sc, cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), None, radiance=True,
                          philox=True, threads=8)
    d = (rp[..., :3].astype(np.float64) - rx[..., :3].astype(np.float64)).reshape(-1, 3)
    se = d.std(axis=0) / math.sqrt(d.shape[0])
    assert np.all(np.abs(d.mean(axis=0)) < 4 * se), (d.mean(axis=0), se)
    assert not np.array_equal(rp, rx)
    assert abs(cp.rays / cx.rays - 1.0) < 0.02  # same path-length distribution
    # frames are independent draws: frame 1 differs from frame 0
    _, rp1, _ = po.render(sc, cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), None, radiance=True,
                          philox=True, frame=1, threads=8)
    assert not np.array_equal(rp1, rp)


def _rgb(pos, cfg):
    return pos.view(np.uint8).reshape(cfg.height, cfg.width, 4)[..., :3].astype(np.float64)


def test_philox_mode_meets_the_psnr_contract():
    """SURVEY.md §8(c) C3, perf mode: PSNR >= 30 dB against a 1024-spp reference at low resolution.  RTIOW at
    64x36: the Philox image at 64 spp (measured 36.1 dB) against the parity mode (cuRAND XORWOW) at 1024 spp.  (The
    kernel's Philox mode equals this oracle's bit for bit: tests/test_gpu_parity.py.)"""
    ref_cfg = scenes.CONFIGS["c2"].scaled(64, 36, 1024)
    cfg = scenes.CONFIGS["c2"].scaled(64, 36, 64)
    sc = po.OracleScene(scenes.builtin(cfg.scene))
    ref, _, _ = po.render(sc, ref_cfg.width, ref_cfg.height, ref_cfg.spp, ref_cfg.depth, ref_cfg.inputs(),
                          po.init_states(ref_cfg.width, ref_cfg.height), threads=8)
    ph, _, _ = po.render(sc, cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), None, philox=True, threads=8)
    mse = ((_rgb(ref, ref_cfg) - _rgb(ph, cfg)) ** 2).mean()
    assert 10 * math.log10(255.0 ** 2 / mse) >= 30.0


def test_philox_mode_estimates_the_cornell_image():
    """The Cornell box (config 3's scene, emissive, depth 16) at 64x64, 64 spp: per channel, the image mean of
    (philox - xorwow) pre-gamma radiance within 3 standard errors (3 sigma; measured 1.3-1.5),
    and the same path-length distribution (ray counts within 1 %).  Cornell at 1024 spp is itself too noisy for a
    PSNR bound (21 dB between 256 and 1024 spp), hence the mean test."""
    cfg = scenes.CONFIGS["c3"].scaled(64, 64, 64)
    sc = po.OracleScene(scenes.builtin(cfg.scene))
    _, rx, cx = po.render(sc, cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(),
                          po.init_states(cfg.width, cfg.height), radiance=True, threads=8)
    _, rp, cp = po.render(sc, cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), None, radiance=True,
                          philox=True, threads=8)
    d = (rp[..., :3].astype(np.float64) - rx[..., :3].astype(np.float64)).reshape(-1, 3)
    se = d.std(axis=0) / math.sqrt(d.shape[0])
    assert np.all(np.abs(d.mean(axis=0)) < 3 * se), (d.mean(axis=0), se)
    assert abs(cp.rays / cx.rays - 1.0) < 0.01


def test_sphere_uv_acos_atan2_are_accurate_and_ieee_signed():
    """GetSphereUV's acos / atan2 (fixed binary32 sequences shared by kernel and oracle, rt_oracle.c): within
    3 ulp of the double-precision functions, with IEEE atan2's signed-zero quadrants."""
    import ctypes as C
    L = po.lib()
    L.orc_acos.restype, L.orc_acos.argtypes = C.c_float, [C.c_float]
    L.orc_atan2.restype, L.orc_atan2.argtypes = C.c_float, [C.c_float, C.c_float]
    rng = np.random.default_rng(7)
    xs = np.concatenate([rng.uniform(-1, 1, 20000), [-1.0, -0.5, 0.0, 0.5, 1.0]]).astype(np.float32)
    got = np.array([L.orc_acos(float(x)) for x in xs], np.float32)
    want = np.arccos(xs.astype(np.float64))
    assert np.all(np.abs(got - want) <= 3 * np.spacing(want.astype(np.float32)))
    assert L.orc_acos(1.0000001) == 0.0 and L.orc_acos(-1.0000001) == np.float32(np.pi)  # clamped
    ys, x2 = rng.normal(size=(2, 20000)).astype(np.float32)
    got = np.array([L.orc_atan2(float(y), float(x)) for y, x in zip(ys, x2)], np.float32)
    want = np.arctan2(ys.astype(np.float64), x2.astype(np.float64))
    assert np.all(np.abs(got - want) <= 3 * np.spacing(np.abs(want).astype(np.float32)))
    pi = np.float32(np.pi)
    assert [L.orc_atan2(-0.0, -1.0), L.orc_atan2(0.0, -1.0), L.orc_atan2(0.0, -0.0)] == [-pi, pi, pi]
    assert np.signbit(L.orc_atan2(-0.0, 1.0)) and L.orc_atan2(0.0, 0.0) == 0.0


def test_native_cpu_baseline_build_computes_the_checker_bits(tmp_path):
    """The CPU baseline (oracle at -O3 -march=native, still without FP contraction) renders
    exactly the checker build's image, so the baseline times the same computation."""
    L = po.native_lib(str(tmp_path / "native"))
    cfg = scenes.CONFIGS["c2"].scaled(64, 40, 4)
    sc = scenes.builtin(cfg.scene)
    st_a, st_b = po.init_states(cfg.width, cfg.height), po.init_states(cfg.width, cfg.height)
    a, _, ca = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st_a)
    b, _, cb = po.render(po.OracleScene(sc, library=L), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st_b,
                         library=L, threads=4)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(st_a, st_b)
    assert ca.rays == cb.rays


def test_flop_model_prices_rectangle_and_sphere_tests_apart():
    """SURVEY §8(d) D4 prices a rectangle test at 12 FLOP and a sphere test at 23.  The oracle counts the rectangle
    tests among its primitive tests (orc_counters.rect_tests); on the C3 golden (Cornell box: 6 rectangles and 2
    spheres, builtin_scenes.cpp cornell) the exact closest-hit scan — what the flat kernels execute — tests every
    primitive per ray, so the split is exactly 6 : 2 per ray, and bench.py's model applies 12 and 23 to it."""
    import bench

    case = CASE_BY_NAME["c3_cornell_128_s16"]
    cfg = case.cfg()
    sc = scenes.builtin(cfg.scene)
    kinds = [int(h.type) for h in sc.hittables]
    n_rect = sum(1 for k in kinds if k != abi.RT_SPHERE)
    assert (n_rect, len(kinds) - n_rect) == (6, 2)
    inp = cfg.inputs()
    st = po.init_states(cfg.width, cfg.height)
    _, _, cnt = po.render(po.OracleScene(sc, exact=True), cfg.width, cfg.height, cfg.spp, cfg.depth, inp, st)
    assert cnt.prim_tests == 8 * cnt.rays and cnt.rect_tests == 6 * cnt.rays
    c = [cnt.rays, cnt.box_tests, cnt.prim_tests, cnt.primary] + [0] * 12 + [cnt.rect_tests] + [0] * 7
    assert len(c) == abi.COUNTERS_WORDS
    want = 21 * cnt.box_tests + 23 * 2 * cnt.rays + 12 * 6 * cnt.rays + 60 * cnt.rays + 40 * cnt.primary
    assert bench.flop_model(c) == want
    # 60 + 2·23 + 6·12 = 178 FLOP per ray plus the camera rays' share (every prim tested at 23 would be 244)
    assert bench.flop_model(c) / cnt.rays == pytest.approx(178 + 40 * cnt.primary / cnt.rays)
    # the reference BVH (golden counters) tests a subset; its rectangle tests are a part of its primitive tests
    st = po.init_states(cfg.width, cfg.height)
    _, _, ref = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, inp, st)
    assert [ref.rays, ref.box_tests, ref.prim_tests, ref.primary] == [int(x) for x in load_golden(case.name)["counters"]]
    assert 0 < ref.rect_tests < ref.prim_tests


def test_philox_mode_dim_scene_bias_is_bounded():
    """The Philox mode sums each sample's channel rounded to the nearest multiple of 2^-12 (include/rt_hip.h
    RT_FLAG_RNG_PHILOX; quant12 in render.hip, orc_quant here), so a sample contributes its value within 2^-13, and a
    positive value below 2^-13 contributes 0.  In a dim scene (RTIOW under a sky 1/256 as bright: most samples carry
    a few 2^-12 or less) the per-channel image mean of (philox - xorwow) pre-gamma radiance stays within 4 standard
    errors plus the rounding's 2^-13 bound (the low-end energy the fixed point loses is bounded and tested)."""
    cfg = scenes.CONFIGS["c2"].scaled(96, 54, 32)
    inp = cfg.inputs()
    for i in range(3):
        inp.background_start[i] = inp.background_start[i] / 256.0
        inp.background_end[i] = inp.background_end[i] / 256.0
    sc = po.OracleScene(scenes.builtin(cfg.scene))
    _, rx, _ = po.render(sc, cfg.width, cfg.height, cfg.spp, cfg.depth, inp, po.init_states(cfg.width, cfg.height),
                         radiance=True, threads=8)
    _, rp, _ = po.render(sc, cfg.width, cfg.height, cfg.spp, cfg.depth, inp, None, radiance=True, philox=True,
                         threads=8)
    x = rx[..., :3].astype(np.float64).reshape(-1, 3)
    p = rp[..., :3].astype(np.float64).reshape(-1, 3)
    assert 0.0 < x.mean() < 8.0 / 4096  # dim: the mean sample is a few quanta (measured 4.5)
    d = p - x
    se = d.std(axis=0) / math.sqrt(d.shape[0])
    assert np.all(np.abs(d.mean(axis=0)) < 4 * se + 2.0 ** -13), (d.mean(axis=0), se)
    # every Philox pixel mean is a whole number of quanta over spp (the fixed-point sum), XORWOW's is not
    q = p * 4096.0 * cfg.spp
    assert np.allclose(q, np.round(q), atol=1e-3 * cfg.spp)
