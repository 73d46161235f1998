"""A/B of RT_TUNE_PIXEL_SORT (v3): each 16x16 region's pixels rendered in the previous launch's ray-count order
(four waves per region, costliest pixels first) against plain 8x8 tiles.  Timed in alternating blocks of frames
(each block's first frame is untimed); frames do not advance the RNG state, so both must render identical bits."""
import argparse, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer

RT_TUNE_PIXEL_SORT = 7
ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--rng", default="xorwow")
ap.add_argument("--blocks", type=int, default=3)
ap.add_argument("--frames", type=int, default=4)
ap.add_argument("--variant", type=int, default=3)
args = ap.parse_args()
cfg = scenes.CONFIGS[args.config]
lib().rt_set_variant(args.variant)
ds = DeviceScene(scenes.builtin(cfg.scene))
r = Renderer(cfg.width, cfg.height, rng=args.rng)
r.render_init()
inp = cfg.inputs()
ref = None
times = {0: [], 1: []}
for b in range(args.blocks):
    for mode in (0, 1):
        lib().rt_set_tuning(RT_TUNE_PIXEL_SORT, mode)
        for f in range(args.frames + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r.render(ds, cfg.spp, cfg.depth, inp, flags=abi.RT_FLAG_NO_STATE_WRITEBACK, frame=0)
            e1.record()
            torch.cuda.synchronize()
            if f:
                times[mode].append(e0.elapsed_time(e1))
            if ref is None:
                ref = r.pos.clone()
            assert torch.equal(r.pos, ref), f"pixel sort {mode}: image differs"
lib().rt_set_tuning(RT_TUNE_PIXEL_SORT, 1)
for mode, t in times.items():
    print(f"{args.config} {args.rng} variant {args.variant} pixel_sort {mode}: median {statistics.median(t):.2f} ms "
          f"min {min(t):.2f} ({len(t)} frames)", flush=True)
