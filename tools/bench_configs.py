"""Per-config timings beyond the headline (BASELINE configs 3, 4 and 5): ms/frame and Mray/s on one GPU.

c3: 3840x2160, 256 spp, depth 16, Cornell box (one frame).
c4: 7680x4320, 128 spp, depth 8, RTIOW: the share of rank 0 of 8 (block-cyclic 16-row bands, 270 of the
    4320 rows), i.e. the work one GPU of the 8-GPU configuration renders per frame; the gather is not
    included (one RCCL gather of 16.6 MB per rank).
c5: 1920x1080, 1 spp, depth 4, textured spheres with three 8192x4096 textures (RGB8, or RGBA8-padded with
    --texel-layouts 4), progressive accumulation with the scripted moving camera (accumulation resets when the
    camera moves; here every frame moves, as in an interactive orbit).
Each config runs with the reference's XORWOW state (parity mode) and with the stateless Philox streams.
"""
import argparse, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer

ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="-1", help="kernel variants to time (rt_set_variant), comma-separated")
ap.add_argument("--configs", default="c3,c4,c5")
ap.add_argument("--rngs", default="xorwow,philox")
ap.add_argument("--texel-layouts", default="3,4", help="c5: device bytes per texel (RT_TUNE_TEXEL_LAYOUT)")
ap.add_argument("--state-layouts", default="curand",
                help="XORWOW state layouts to time: curand (the reference's 48-B structs), soa (native planes)")
args = ap.parse_args()


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


_scenes = {}


def scene_for(config, layout):
    key = (config, layout)
    if key not in _scenes:
        prev = lib().rt_set_tuning(6, layout)
        _scenes[key] = DeviceScene(scenes.CONFIGS[config].scene_desc())
        lib().rt_set_tuning(6, prev)
    return _scenes[key]


def run(variant, config, rng, layout=3, state_layout="curand"):
    lib().rt_set_variant(variant)
    cfg = scenes.CONFIGS[config]
    ds = scene_for(config, layout)
    out = {"config": config, "rng": rng, "variant": variant,
           "workload": f"{cfg.width}x{cfg.height}, {cfg.spp} spp, depth {cfg.depth}"}
    if rng == "xorwow":
        out["state_layout"] = state_layout
    if config == "c5":
        out["texel_bytes"] = layout
        out["texture_size"] = list(cfg.texture_size)
    if config == "c5":
        r = Renderer(cfg.width, cfg.height, rng=rng, state_layout=state_layout)
        r.render_init()
        frames, times = 60, []
        r.counters.zero_()
        for f in range(frames):
            pos, fwd = scenes.moving_camera(f, frames)
            inp = scenes.camera_inputs(pos, fwd, cfg.fov)
            r.reset_accumulation()
            times.append(timed(lambda: r.render(ds, cfg.spp, cfg.depth, inp, flags=abi.RT_FLAG_ACCUMULATE)))
        rays = int(r.counters[0])
        out.update(ms_per_frame_median=round(sorted(times)[len(times) // 2], 3), frames=frames, rays=rays,
                   Mray_per_s=round(rays / sum(times) / 1e3, 1))
        return out
    kw = {}
    if config == "c4":
        kw = dict(band_rows=16, num_ranks=8, rank=0)
        out["workload"] += ", rank 0 of 8 (16-row bands)"
    r = Renderer(cfg.width, cfg.height, rng=rng, state_layout=state_layout, **kw)
    r.render_init()
    r.render(ds, 1, cfg.depth, cfg.inputs())  # warm-up
    torch.cuda.synchronize()
    r.counters.zero_()
    ms = timed(lambda: r.render(ds, cfg.spp, cfg.depth, cfg.inputs()))
    rays = int(r.counters[0])
    out.update(ms_per_frame=round(ms, 2), rays=rays, Mray_per_s=round(rays / ms / 1e3, 1))
    return out


for v in (int(x) for x in args.variants.split(",")):
    for config in args.configs.split(","):
        for rng in args.rngs.split(","):
            for layout in ([int(x) for x in args.texel_layouts.split(",")] if config == "c5" else [3]):
                for sl in (args.state_layouts.split(",") if rng == "xorwow" else ["curand"]):
                    print(json.dumps(run(v, config, rng, layout, sl)), flush=True)
