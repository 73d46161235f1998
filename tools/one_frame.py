"""Render N frames of a config with one kernel variant (for rocprofv3 runs)."""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--variant", type=int, default=-1)
ap.add_argument("--frames", type=int, default=2)
ap.add_argument("--rng", default="xorwow", choices=("xorwow", "philox"))
ap.add_argument("--state-layout", default="curand", choices=("curand", "soa"))
ap.add_argument("--lds-pad", type=int, default=0)
ap.add_argument("--texel-bytes", type=int, default=3, help="RT_TUNE_TEXEL_LAYOUT (3 = RGB8, 4 = RGBA8)")
args = ap.parse_args()
cfg = scenes.CONFIGS[args.config]
lib().rt_set_variant(args.variant)
lib().rt_set_tuning(4, args.lds_pad)
lib().rt_set_tuning(6, args.texel_bytes)
ds = DeviceScene(cfg.scene_desc())  # c5: three 8192x4096 textures
r = Renderer(cfg.width, cfg.height, rng=args.rng, state_layout=args.state_layout)
r.render_init()
flags = abi.RT_FLAG_ACCUMULATE if args.config == "c5" else 0
for f in range(args.frames):
    inp = cfg.inputs()
    if args.config == "c5":  # as bench.py renders C5: the scripted orbit, the accumulation restarted per frame
        pos, fwd = scenes.moving_camera(f, 60)
        inp = scenes.camera_inputs(pos, fwd, cfg.fov)
        r.reset_accumulation()
    r.render(ds, cfg.spp, cfg.depth, inp, flags=flags)
torch.cuda.synchronize()
print("rays/frame", int(r.counters[0]) // args.frames)
