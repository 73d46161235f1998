"""C5: does a cost-ordered work queue shorten the persistent flat kernel's tail?  

Each C5 frame (1920x1080, 1 spp, depth 4, moving camera, accumulation restarted) records per pixel the loop passes it
took (rt_set_pixel_cost).  The next frame's queue hands the 8x8 tiles out costliest first (rt_set_tile_order: the tiles
sorted by the previous frame's summed passes, dealt round-robin over the 16 queue heads so every head's range runs from
its costliest tile to its cheapest).  Compared with the row-major queue on the same camera path, XORWOW and Philox.
The plan is computed on the host here: this measures the schedule's gain before a device-side planner is built.

  python tools/c5_order.py [--frames 16]
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

HEADS = 16  # kQueueCounters (render.hip)

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=16)
ap.add_argument("--variant", type=int, default=6)
ap.add_argument("--depths", default="4")
args = ap.parse_args()

c5 = scenes.CONFIGS["c5"]
ds5 = DeviceScene(c5.scene_desc())
tiles_x, tiles_y = (c5.width + 7) // 8, (c5.height + 7) // 8
tiles = tiles_x * tiles_y
T = (tiles + HEADS - 1) // HEADS
positions = np.array([j * T + s for s in range(T) for j in range(HEADS) if j * T + s < tiles], np.int64)
cost = torch.zeros(tiles * 64, dtype=torch.uint8, device="cuda")


def plan(cost_bytes: np.ndarray, order: np.ndarray | None) -> np.ndarray:
    per_slot = cost_bytes.reshape(tiles, 64).astype(np.int64).sum(axis=1)
    tile_cost = np.empty(tiles, np.int64)
    tile_cost[order if order is not None else np.arange(tiles)] = per_slot
    ranked = np.argsort(-tile_cost, kind="stable")
    out = np.empty(tiles, np.uint32)
    out[positions] = ranked
    return out


def run(depth, rng, mode):
    lib().rt_set_variant(args.variant)
    r = Renderer(c5.width, c5.height, rng=rng, state_layout="soa")
    r.render_init()
    lib().rt_set_timing(1)
    order = None
    order_dev = None
    ms = []
    for f in range(args.frames + 2):
        pos, fwd = scenes.moving_camera(f, 60)
        r.reset_accumulation()
        lib().rt_set_pixel_cost(cost.data_ptr(), cost.numel())
        lib().rt_set_tile_order(order_dev.data_ptr() if order_dev is not None else None)
        r.render(ds5, c5.spp, depth, scenes.camera_inputs(pos, fwd, c5.fov), flags=abi.RT_FLAG_ACCUMULATE)
        torch.cuda.synchronize()
        if f >= 2:
            ms.append(lib().rt_last_kernel_ms())
        if mode == "ordered":
            order = plan(cost.cpu().numpy(), order)
            order_dev = torch.from_numpy(order.view(np.int32)).cuda()
    lib().rt_set_pixel_cost(None, 0)
    lib().rt_set_tile_order(None)
    lib().rt_set_timing(0)
    lib().rt_set_variant(-1)
    img = r.image()
    return float(np.median(ms)), float(np.min(ms)), img


for depth in (int(d) for d in args.depths.split(",")):
    for rng in ("xorwow", "philox"):
        base, base_min, img0 = run(depth, rng, "rowmajor")
        ordd, ord_min, img1 = run(depth, rng, "ordered")
        same = np.array_equal(img0, img1)
        print(f"depth {depth} {rng:7s}: row-major {base:.3f} ms (min {base_min:.3f}), cost-ordered {ordd:.3f} ms "
              f"(min {ord_min:.3f}): {100 * (ordd / base - 1):+.1f} %; same last image: {same}", flush=True)
