"""Rays per frame whose closest hit the exactness check sends through the reference BVH (counters[17] of a
RT_FLAG_COUNT_TESTS launch: render.hip bvh_clear / bvh_replay for the BVH kernels, flat_trace for the flat ones), per
config and kernel variant, with the frame time of the product build beside it.
    python tools/replay_rate.py --configs c2,c4,c3 --variants -1,3,4"""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer

ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="c2")
ap.add_argument("--variants", default="-1")
ap.add_argument("--rng", default="xorwow", choices=("xorwow", "philox"))
ap.add_argument("--spp", type=int, default=0, help="override the config's samples per pixel (0: as configured)")
args = ap.parse_args()
for name in args.configs.split(","):
    cfg = scenes.CONFIGS[name]
    if args.spp:
        cfg = cfg.scaled(cfg.width, cfg.height, args.spp)
    ds = DeviceScene(cfg.scene_desc())
    r = Renderer(cfg.width, cfg.height, rng=args.rng)
    r.render_init()
    for v in (int(x) for x in args.variants.split(",")):
        lib().rt_set_variant(v)
        r.counters.zero_()
        r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_COUNT_TESTS | abi.RT_FLAG_NO_STATE_WRITEBACK)
        torch.cuda.synchronize()
        rays, replays = int(r.counters[0]), int(r.counters[17])
        lib().rt_set_timing(1)
        r.render(ds, cfg.spp, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_NO_STATE_WRITEBACK)
        torch.cuda.synchronize()
        ms = lib().rt_last_kernel_ms()
        lib().rt_set_timing(0)
        print(json.dumps({"config": name, "variant": lib().rt_last_variant(), "rng": args.rng, "rays": rays,
                          "replays": replays, "replay_rate": replays / max(rays, 1), "kernel_ms": round(ms, 3)}),
              flush=True)
