"""Frame time of a scene the automatic choice keeps on the flat kernels for exactness (tests/adversarial_scene.py's
20-primitive scene, touching rectangles) against the BVH kernel it would otherwise run: 1920x1080, 64 spp, depth 8."""
import os, statistics, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import torch
from adversarial_scene import ADVERSARIAL_CONFIG, adversarial_scene_large
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer

cfg = ADVERSARIAL_CONFIG.scaled(1920, 1080, 64)
ds = DeviceScene(adversarial_scene_large())
r = Renderer(cfg.width, cfg.height)
r.render_init()
times = {3: [], 5: [], -1: []}
for rnd in range(4):
    for v in times:
        lib().rt_set_variant(v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r.render(ds, cfg.spp, 8, cfg.inputs())
        e1.record()
        torch.cuda.synchronize()
        if rnd:
            times[v].append(e0.elapsed_time(e1))
        if v == -1 and rnd == 3:
            print("automatic choice ran variant", lib().rt_last_variant())
for v, t in times.items():
    print(f"variant {v}: median {statistics.median(t):.3f} ms", flush=True)
