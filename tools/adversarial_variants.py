"""Pixels of the adversarial scene (tests/adversarial_scene.py) that each kernel variant renders differently from the
oracle's reference traversal (diagnostic: the BVH kernels are not expected to match on ties and box-face hits)."""
import sys, numpy as np, torch
import os; R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, 'tests'))
from adversarial_scene import ADVERSARIAL_CONFIG, adversarial_scene
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer
from oracle import py_oracle as po
cfg, sc = ADVERSARIAL_CONFIG, adversarial_scene()
st = po.init_states(cfg.width, cfg.height)
ref, _, _ = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st)
for v in (2, 3, 4, 5, 6):
    lib().rt_set_variant(v)
    r = Renderer(cfg.width, cfg.height); r.render_init()
    r.render(DeviceScene(sc), cfg.spp, cfg.depth, cfg.inputs()); torch.cuda.synchronize()
    print('variant', v, 'pixels differing from the reference traversal:', int((r.image() != ref).sum()), flush=True)
