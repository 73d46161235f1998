"""Where a flat-kernel (variant 5) frame's wave time goes, from its COUNT_TESTS build: wave cycles in the trace
(the primitive scan and the exactness check), in shading (camera rays included) and in the camera-ray code, and the
lanes each phase serves per pass.  One frame per config, RNG state not written back.
    python tools/flat_phases.py [--configs c3,c1] [--spp N]"""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer

ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="c3")
ap.add_argument("--spp", type=int, default=0, help="override the config's spp (0: as configured)")
ap.add_argument("--variant", type=int, default=5)
args = ap.parse_args()
for name in args.configs.split(","):
    cfg = scenes.CONFIGS[name]
    ds = DeviceScene(cfg.scene_desc())
    r = Renderer(cfg.width, cfg.height, rng=os.environ.get("RT_RNG", "xorwow"))
    r.render_init()
    lib().rt_set_variant(args.variant)
    r.counters.zero_()
    inp = cfg.inputs() if name != "c5" else scenes.camera_inputs(*scenes.moving_camera(0, 60), cfg.fov)
    r.render(ds, args.spp or cfg.spp, cfg.depth, inp, flags=abi.RT_FLAG_COUNT_TESTS | abi.RT_FLAG_NO_STATE_WRITEBACK)
    torch.cuda.synchronize()
    c = [int(x) for x in r.counters.tolist()]
    rays, passes, shades = c[0], c[4], c[6]
    trav, shade, total, cam = c[7], c[8], c[9], c[5]
    lt, ls, lc = c[13], c[14], c[15]
    print(f"{name} variant {args.variant}: {rays} rays, {passes} wave passes ({64 * passes / rays:.2f} per 64 rays) | "
          f"wave time: trace {trav / total:.3f} shade {(shade - cam) / total:.3f} camera {cam / total:.3f} "
          f"other {(total - trav - shade) / total:.3f} | lanes per pass: tracing {lt / passes:.1f} "
          f"shading {ls / passes:.1f} starting a sample {lc / passes:.1f} | cycles per pass {total / passes:.0f}: "
          f"trace {trav / passes:.0f} shade {(shade - cam) / passes:.0f} camera {cam / passes:.0f}", flush=True)
lib().rt_set_variant(-1)
