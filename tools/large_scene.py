"""Frame time of large scenes (the viewer's AddHittable grows scenes without limit,
CudaLayer.cpp:918-1370) at config 2's frame (1920x1080, 64 spp, depth 8, C2 camera) over sphere fields of
N spheres: the 16- or 32-bit-reference v3 / v4 kernels against the v2 / v1 kernels they replaced as the
fallback beyond 16-bit references.  One warm frame, then the median of --frames timed frames (HIP events)."""
import argparse, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cudaraytracer_amd import scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer

ap = argparse.ArgumentParser()
ap.add_argument("--n", default="6000,9000,20000,60000")
ap.add_argument("--variants", default="3,4,1,0")
ap.add_argument("--frames", type=int, default=3)
ap.add_argument("--spp", type=int, default=64)
args = ap.parse_args()
cfg = scenes.CONFIGS["c2"]
for n in (int(x) for x in args.n.split(",")):
    ds = DeviceScene(scenes.sphere_field(n, 11))
    info = ds.info()
    for v in (int(x) for x in args.variants.split(",")):
        lib().rt_set_variant(v)
        r = Renderer(cfg.width, cfg.height, state_layout="soa")
        r.render_init()
        r.render(ds, args.spp, cfg.depth, cfg.inputs())
        torch.cuda.synchronize()
        ms = []
        r.counters.zero_()
        for _ in range(args.frames):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r.render(ds, args.spp, cfg.depth, cfg.inputs())
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        rays = int(r.counters[0]) / args.frames
        med = sorted(ms)[len(ms) // 2]
        print(json.dumps({"spheres": n, "nodes": info.num_nodes, "bvh_depth": info.bvh_depth, "variant": v,
                          "launched": lib().rt_last_variant(), "ms_per_frame": round(med, 3),
                          "Mray_s": round(rays / med / 1e3, 1), "spp": args.spp}), flush=True)
        del r
lib().rt_set_variant(-1)
