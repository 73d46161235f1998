"""C5: per-work-index pass counts of a few frames of the orbit (rt_set_pixel_cost), for tools/c5_sched_sim.py.

Each C5 frame (1920x1080, 1 spp, depth 4, moving camera, accumulation restarted) is rendered on the persistent flat
kernel (variant 6) with the pixel-cost buffer set: byte i = the loop passes work index i took from its start to its
pixel write.  Saved as uint8[frames, work_total] to gpurun_out/c5_cost.npz with the work-index geometry.

  python tools/c5_cost_dump.py [--frames 4] [--out gpurun_out/c5_cost.npz]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=4)
ap.add_argument("--out", default="gpurun_out/c5_cost.npz")
args = ap.parse_args()

c5 = scenes.CONFIGS["c5"]
ds = DeviceScene(c5.scene_desc())
tiles = ((c5.width + 7) // 8) * ((c5.height + 7) // 8)
cost = torch.zeros(tiles * 64, dtype=torch.uint8, device="cuda")
lib().rt_set_variant(6)
r = Renderer(c5.width, c5.height, state_layout="soa")
r.render_init()
lib().rt_set_timing(1)
out, ms = [], []
for f in range(args.frames + 2):
    pos, fwd = scenes.moving_camera(f, 60)
    cost.zero_()
    lib().rt_set_pixel_cost(cost.data_ptr(), cost.numel())
    r.render(ds, c5.spp, c5.depth, scenes.camera_inputs(pos, fwd, c5.fov), flags=abi.RT_FLAG_ACCUMULATE)
    torch.cuda.synchronize()
    if f >= 2:
        out.append(cost.cpu().numpy().copy())
        ms.append(lib().rt_last_kernel_ms())
lib().rt_set_pixel_cost(None, 0)
lib().rt_set_timing(0)
lib().rt_set_variant(-1)
os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
np.savez_compressed(args.out, cost=np.stack(out), kernel_ms=np.array(ms), width=c5.width, height=c5.height)
c = np.stack(out).astype(np.float64)
print(f"{len(out)} frames, kernel ms {np.round(ms, 4).tolist()}; passes per pixel mean {c.mean():.3f}, "
      f"p50/90/99/max {np.percentile(c, [50, 90, 99]).tolist()} / {c.max():.0f}", flush=True)
