"""Philox C3 128x128 case per kernel variant: pixels and rays that differ from the oracle's reference traversal
(exact=False) and from its brute-force closest hit (exact=True)."""
import sys, os
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import numpy as np, torch
from cases import CASE_BY_NAME
from cudaraytracer_amd import scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer
from oracle import py_oracle as po
case = CASE_BY_NAME["c3_cornell_128_s16"]; cfg = case.cfg(); sc = scenes.builtin(cfg.scene)
refs = {}
for exact in (False, True):
    refs[exact] = po.render(po.OracleScene(sc, exact=exact), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), None,
                            faithful_grid=case.faithful_grid, rius_order=case.rius_order, philox=True, seed=1984, frame=5)
for v in (2, 3, 4, 5, 6):
    lib().rt_set_variant(v)
    r = Renderer(cfg.width, cfg.height, rng="philox"); r.render_init()
    r.render(DeviceScene(sc), cfg.spp, cfg.depth, cfg.inputs(), flags=case.flags, frame=5); torch.cuda.synchronize()
    img = r.image(); rays = int(r.counters[0])
    print(v, {e: (int((img != refs[e][0]).sum()), rays - refs[e][2].rays) for e in refs}, flush=True)
