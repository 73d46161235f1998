"""Per-config timings beyond the headline (BASELINE configs 3 and 5): ms/frame and Mray/s on one GPU.

c3: 3840x2160, 256 spp, depth 16, Cornell box (one frame).
c5: 1920x1080, 1 spp, depth 4, textured spheres, progressive accumulation with the scripted moving camera
    (accumulation resets when the camera moves; here every frame moves, as in an interactive orbit).
"""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd.renderer import DeviceScene, Renderer

out = {}
cfg = scenes.CONFIGS["c3"]
ds = DeviceScene(scenes.builtin(cfg.scene))
r = Renderer(cfg.width, cfg.height)
r.render_init()
r.render(ds, 1, cfg.depth, cfg.inputs())  # warm-up
torch.cuda.synchronize()
r.counters.zero_()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); r.render(ds, cfg.spp, cfg.depth, cfg.inputs()); e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1); rays = int(r.counters[0])
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
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); r.render(ds, cfg.spp, cfg.depth, inp, flags=abi.RT_FLAG_ACCUMULATE); e1.record()
    torch.cuda.synchronize()
    times.append(e0.elapsed_time(e1))
rays = int(r.counters[0])
ms = sorted(times)[len(times) // 2]
out["c5"] = {"ms_per_frame_median": round(ms, 3), "frames": frames, "rays": rays,
             "Mray_per_s": round(rays / sum(times) / 1e3, 1)}
print(json.dumps(out))
