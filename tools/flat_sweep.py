"""Interleaved same-process timing of the flat kernels against the BVH kernels on small scenes, and of the flat
kernels' RandomInUnitSphere cap (RT_TUNE_RIUS_TRIPS).  Frames advance their RNG states as bench.py's do.
    python tools/flat_sweep.py [--configs c1,default,c3] [--trips 2,3,4,6] [--rounds 3]"""
import argparse, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer

ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="c1,default,c3")
ap.add_argument("--trips", default="4")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--rng", default="xorwow")
args = ap.parse_args()
lib().rt_set_tuning(abi.RT_TUNE_FLAT_MAX, 64)
for name in args.configs.split(","):
    cfg = scenes.CONFIGS[name]
    ds = DeviceScene(cfg.scene_desc())
    r = Renderer(cfg.width, cfg.height, rng=args.rng)
    r.render_init()
    inp = cfg.inputs() if name != "c5" else scenes.camera_inputs(*scenes.moving_camera(0, 60), cfg.fov)
    runs = [(3, 0)] + [(5, int(k)) for k in args.trips.split(",")] + [(4, 0), (6, 4)]
    times = {k: [] for k in runs}
    for rnd in range(args.rounds + 1):
        for v, k in runs:
            lib().rt_set_variant(v)
            lib().rt_set_tuning(abi.RT_TUNE_RIUS_TRIPS, k)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r.render(ds, cfg.spp, cfg.depth, inp)
            e1.record()
            torch.cuda.synchronize()
            if rnd:  # (round 0 warms every kernel and builds the tile orders)
                times[(v, k)].append(e0.elapsed_time(e1))
    for (v, k), t in times.items():
        print(f"{name} ({ds.info().num_primitives} prims, {cfg.width}x{cfg.height} {cfg.spp} spp depth {cfg.depth}) "
              f"variant {v} trips {k}: median {statistics.median(t):.3f} ms  min {min(t):.3f}", flush=True)
lib().rt_set_variant(-1)
