"""Per-config timings beyond the headline (BASELINE configs 3 and 5): ms/frame and Mray/s on one GPU.

c3: 3840x2160, 256 spp, depth 16, Cornell box (one frame).
c5: 1920x1080, 1 spp, depth 4, textured spheres, progressive accumulation with the scripted moving camera
    (accumulation resets when the camera moves; here every frame moves, as in an interactive orbit).
"""
import argparse, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer

ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="-1", help="kernel variants to time (rt_set_variant), comma-separated")
args = ap.parse_args()


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def run(variant):
    lib().rt_set_variant(variant)
    out = {"variant": variant}
    cfg = scenes.CONFIGS["c3"]
    ds = DeviceScene(scenes.builtin(cfg.scene))
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    r.render(ds, 1, cfg.depth, cfg.inputs())  # warm-up
    torch.cuda.synchronize()
    r.counters.zero_()
    ms = timed(lambda: r.render(ds, cfg.spp, cfg.depth, cfg.inputs()))
    rays = int(r.counters[0])
    out["c3"] = {"ms_per_frame": round(ms, 2), "rays": rays, "Mray_per_s": round(rays / ms / 1e3, 1)}
    del r
    cfg = scenes.CONFIGS["c5"]
    ds = DeviceScene(scenes.builtin(cfg.scene))
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    frames = 60
    times = []
    r.counters.zero_()
    for f in range(frames):
        pos, fwd = scenes.moving_camera(f, frames)
        inp = scenes.camera_inputs(pos, fwd, cfg.fov)
        r.reset_accumulation()
        times.append(timed(lambda: r.render(ds, cfg.spp, cfg.depth, inp, flags=abi.RT_FLAG_ACCUMULATE)))
    rays = int(r.counters[0])
    ms = sorted(times)[len(times) // 2]
    out["c5"] = {"ms_per_frame_median": round(ms, 3), "frames": frames, "rays": rays,
                 "Mray_per_s": round(rays / sum(times) / 1e3, 1)}
    return out


for v in (int(x) for x in args.variants.split(",")):
    print(json.dumps(run(v)), flush=True)
