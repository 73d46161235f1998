"""Regenerate the golden fixtures in tests/golden/ from the CPU oracle (oracle/rt_oracle.c).

    python tests/golden/make_golden.py

Inputs are the built-in scenes of librt_hip.so's host code (csrc/builtin_scenes.cpp; no device needed) and
the BASELINE configurations of cudaraytracer_amd/scenes.py; outputs are the oracle's RGBA8 images, RNG
states after the frame and ray/test counters.  Scene tables are stored too, so a change of the scene
generators shows up as a fixture mismatch.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from cases import CASES, PHILOX_CASES  # noqa: E402
from cudaraytracer_amd import abi, scenes  # noqa: E402
from oracle import py_oracle as po  # noqa: E402


def xorwow_kat() -> dict:
    out = {}
    for seed in (0, 1, 1984, 1985, 1984 + 1919, (1 << 32) + 7, 2**63 + 12345):
        st = abi.CurandState()
        po.lib().orc_curand_init(seed, C.byref(st))
        init = [st.d] + list(st.v)
        raw = [po.lib().orc_curand(C.byref(st)) for _ in range(8)]
        po.lib().orc_curand_init(seed, C.byref(st))
        uni = [float(po.lib().orc_curand_uniform(C.byref(st))) for _ in range(8)]
        out[str(seed)] = {"init": init, "raw": raw, "uniform": uni}
    return out


def digest(a: np.ndarray) -> bytes:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()


def row_digests(a: np.ndarray) -> np.ndarray:
    """SHA-256 of each row of a (H, ...) array: (H, 32) uint8."""
    return np.stack([np.frombuffer(digest(r), np.uint8) for r in a])


def c4_frame_digests(threads: int = 8) -> None:
    """BASELINE config 4's whole frame (7680×4320, 128 spp, depth 8, RTIOW, XORWOW, Random() right to left, one
    rank) from the oracle's reference traversal: per row the SHA-256 of its RGBA8 pixels and of its pixels' advanced
    RNG words (d, v[0..4]), and the frame's ray count — 276 KB instead of 133 MB of image and 800 MB of state
    (tests/test_gpu_configs.py::test_c4_whole_frame_row_digests; ~3 min on 8 threads)."""
    cfg = scenes.CONFIGS["c4"]
    sc = scenes.builtin(cfg.scene)
    st = po.init_states(cfg.width, cfg.height)
    pos, _, cnt = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st,
                            threads=threads)
    words = st[:, :6].reshape(cfg.height, cfg.width, 6)
    np.savez_compressed(os.path.join(HERE, "c4_frame_row_digests.npz"),
                        config=np.array([cfg.width, cfg.height, cfg.spp, cfg.depth], np.uint32),
                        pos_row_sha256=row_digests(pos), state_row_sha256=row_digests(words),
                        counters=np.array([cnt.rays, cnt.box_tests, cnt.prim_tests, cnt.primary], np.uint64))
    print("c4", pos.shape, cnt.rays, flush=True)


def main(philox_only: bool = False) -> None:
    if philox_only:  # python tests/golden/make_golden.py --philox-only
        return philox_goldens()
    with open(os.path.join(HERE, "xorwow_kat.json"), "w") as f:
        json.dump(xorwow_kat(), f, indent=1)
    for which in range(5):
        s = scenes.builtin(which)
        np.savez_compressed(os.path.join(HERE, f"scene_{which}.npz"),
                            hittables=np.frombuffer(s.hittables_bytes(), np.uint8),
                            materials=np.frombuffer(s.materials_bytes(), np.uint8))
    for case in CASES:
        cfg = case.cfg()
        sc = scenes.builtin(cfg.scene)
        osc = po.OracleScene(sc)
        inp = cfg.inputs()
        st = po.init_states(cfg.width, cfg.height, full=not case.faithful_grid)
        st0 = st.copy()
        pos, rad, cnt = po.render(osc, cfg.width, cfg.height, cfg.spp, cfg.depth, inp, st,
                                  faithful_grid=case.faithful_grid, rius_order=case.rius_order, radiance=True)
        np.savez_compressed(
            os.path.join(HERE, f"{case.name}.npz"),
            inputs=np.frombuffer(bytes(inp), np.uint8),
            pos=pos,
            # RNG words d, v[0..4] are incompressible: keep digests (tests recompute them)
            state_before_sha256=np.frombuffer(digest(st0[:, :6]), np.uint8),
            state_after_sha256=np.frombuffer(digest(st[:, :6]), np.uint8),
            radiance_sha256=np.frombuffer(digest(rad), np.uint8),
            counters=np.array([cnt.rays, cnt.box_tests, cnt.prim_tests, cnt.primary], np.uint64),
            texture_sha256=np.frombuffer(digest(np.concatenate([np.asarray(i).ravel() for i in sc.images])
                                                if sc.images else np.zeros(0, np.uint8)), np.uint8))
        print(case.name, pos.shape, cnt.rays, flush=True)
    philox_goldens()


def philox_goldens() -> None:
    for case, frame in PHILOX_CASES:
        cfg = case.cfg()
        sc = scenes.builtin(cfg.scene)
        pos, rad, cnt = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), None,
                                  faithful_grid=case.faithful_grid, rius_order=case.rius_order, radiance=True,
                                  philox=True, seed=1984, frame=frame)
        np.savez_compressed(
            os.path.join(HERE, f"philox_{case.name}_f{frame}.npz"),
            inputs=np.frombuffer(bytes(cfg.inputs()), np.uint8), pos=pos,
            radiance_sha256=np.frombuffer(digest(rad), np.uint8),
            counters=np.array([cnt.rays, cnt.box_tests, cnt.prim_tests, cnt.primary], np.uint64))
        print("philox", case.name, frame, cnt.rays, flush=True)


if __name__ == "__main__":
    if "--c4" in sys.argv:  # python tests/golden/make_golden.py --c4   (the whole-frame C4 digests only)
        c4_frame_digests()
    else:
        main(philox_only="--philox-only" in sys.argv)
