"""SIMD efficiency per phase from the COUNT_TESTS wave-iteration counters, for several variants."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer
cfg = scenes.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
ds = DeviceScene(scenes.builtin(cfg.scene))
r = Renderer(cfg.width, cfg.height, rng=os.environ.get("RT_RNG", "xorwow"))
r.render_init()
for v in [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "6,8").split(",")]:
    lib().rt_set_variant(v)
    r.counters.zero_()
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_COUNT_TESTS | abi.RT_FLAG_NO_STATE_WRITEBACK)
    torch.cuda.synchronize()
    c = [int(x) for x in r.counters.tolist()]
    rays, boxes, prims, prim_s, wn, wl, ws = c[0], c[1], c[2], c[3], c[4], c[5], c[6]
    print(f"variant {v}: rays {rays} node-visits/ray {boxes/2/rays:.2f} prim-tests/ray {prims/rays:.2f} | "
          f"SIMD eff: node {boxes/2/(64*wn):.3f} leaf {prims/(64*wl):.3f} shade {rays/(64*ws):.3f} | "
          f"wave-iters per 64 rays: node {64*wn/rays:.1f} leaf {64*wl/rays:.1f} shade {64*ws/rays:.2f} | "
          f"wave time: trace {c[7]/max(1,c[9]):.3f} (leaf {c[10]/max(1,c[9]):.3f}) shade {c[8]/max(1,c[9]):.3f} "
          f"cycles per 64 rays {64*c[9]/rays:.0f} | uniform wave-iters: node {c[11]/max(1,wn):.3f} leaf {c[12]/max(1,wl):.3f} | "
          f"node-iteration lanes: active {boxes/2/wn:.1f} idle: pixel-done {c[13]/max(1,wn):.1f} ray-finished {c[14]/max(1,wn):.1f} "
          f"leaf-waiting {c[15]/max(1,wn):.1f}", flush=True)
