"""Diagnostic (RT_DIAG_OCT build): fraction of v3 node iterations whose tracing lanes share one ray-direction octant
(where an octant-specialised slab test, one FMA per plane distance, would apply), and of those with one node."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer
for name in (sys.argv[1] if len(sys.argv) > 1 else "c2").split(","):
    cfg = scenes.CONFIGS[name]
    ds = DeviceScene(scenes.builtin(cfg.scene))
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    lib().rt_set_variant(3)
    r.counters.zero_()
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_COUNT_TESTS | abi.RT_FLAG_NO_STATE_WRITEBACK)
    torch.cuda.synchronize()
    c = [int(x) for x in r.counters.tolist()]
    print(f"{name}: node iterations {c[4]}, octant-uniform {c[13] / c[4]:.3f}, octant- and node-uniform "
          f"{c[14] / c[4]:.3f}, node-uniform (all) {c[11] / c[4]:.3f}", flush=True)
