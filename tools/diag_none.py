"""Diagnostic (RT_DIAG_NONE build): fraction of node visits whose two children both miss, and of those the
visits caused by the t_best clip alone (what a stored entry distance per stack entry could skip)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer
for name in (sys.argv[1] if len(sys.argv) > 1 else "c2").split(","):
    cfg = scenes.CONFIGS[name]
    ds = DeviceScene(scenes.builtin(cfg.scene))
    r = Renderer(cfg.width, cfg.height, rng="xorwow")
    r.render_init()
    lib().rt_set_variant(3)
    r.counters.zero_()
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_COUNT_TESTS | abi.RT_FLAG_NO_STATE_WRITEBACK)
    torch.cuda.synchronize()
    c = [int(x) for x in r.counters.tolist()]
    visits = c[1] // 2
    print(f"{name}: rays {c[0]} visits/ray {visits / c[0]:.2f} none {c[13] / visits:.3f} "
          f"none-by-t_best {c[14] / visits:.3f} prims/ray {c[2] / c[0]:.2f}", flush=True)
