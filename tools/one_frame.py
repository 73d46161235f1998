"""Render N frames of a config with one kernel variant (for rocprofv3 runs)."""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cudaraytracer_amd import scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--variant", type=int, default=-1)
ap.add_argument("--frames", type=int, default=2)
ap.add_argument("--rng", default="xorwow", choices=("xorwow", "philox"))
ap.add_argument("--lds-pad", type=int, default=0)
args = ap.parse_args()
cfg = scenes.CONFIGS[args.config]
lib().rt_set_variant(args.variant)
lib().rt_set_tuning(4, args.lds_pad)
ds = DeviceScene(scenes.builtin(cfg.scene))
r = Renderer(cfg.width, cfg.height, rng=args.rng)
r.render_init()
for _ in range(args.frames):
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs())
torch.cuda.synchronize()
print("rays/frame", int(r.counters[0]) // args.frames)
