"""C2's ray-coherence ceiling: how much faster does v3's traversal trace a frame's secondary rays
when they are regrouped — the gain a wavefront path tracer would be built for.

1. Render C2's frame (1920x1080, RTIOW, depth 8) at --spp samples on v3 with the ray dump on (rt_set_ray_dump): every
   ray that starts at bounce 1 (the first scattered ray of a path) is appended — generation order, i.e. the order
   v3's waves produce them (8x8 tiles, lanes as their paths reach the bounce).
2. Trace them alone with rt_trace_rays (v3's traversal, no shading) in that order, in a random shuffle, and sorted:
   (a) direction octant, then a 30-bit Morton code of the origin; (b) a Morton code of the direction quantised on the
   unit cube, then the origin's.  Time (HIP events) and the node-loop lane utilisation (box tests / 2 over 64 x wave
   node iterations) per order; the hits must be the same rays' hits in every order.

  python tools/coherence.py --spp 1,4 [--out gpurun_out/coherence.json]
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd._lib import check, lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer

ap = argparse.ArgumentParser()
ap.add_argument("--spp", default="1,4")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--cap", type=int, default=16 << 20)
ap.add_argument("--out", default="gpurun_out/coherence.json")
args = ap.parse_args()

cfg = scenes.CONFIGS["c2"]
ds = DeviceScene(scenes.builtin(cfg.scene))
dev = torch.device("cuda", 0)


def part1by2(v: torch.Tensor) -> torch.Tensor:
    """10-bit integers -> every third bit (Morton interleave helper)."""
    v = v & 0x3FF
    v = (v | (v << 16)) & 0x030000FF
    v = (v | (v << 8)) & 0x0300F00F
    v = (v | (v << 4)) & 0x030C30C3
    v = (v | (v << 2)) & 0x09249249
    return v


def morton3(p: torch.Tensor) -> torch.Tensor:
    lo, hi = p.min(dim=0).values, p.max(dim=0).values
    q = ((p - lo) / torch.clamp(hi - lo, min=1e-20) * 1023.0).clamp(0, 1023).to(torch.int64)
    return part1by2(q[:, 0]) | (part1by2(q[:, 1]) << 1) | (part1by2(q[:, 2]) << 2)


def trace(rays: torch.Tensor, reps: int):
    n = rays.shape[0] // 2
    hits = torch.empty(2 * n, dtype=torch.int32, device=dev)
    cnt = torch.zeros(abi.COUNTERS_WORDS, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    # counting pass
    check(lib().rt_trace_rays(ds.handle, C.c_void_p(rays.data_ptr()), n, C.c_void_p(hits.data_ptr()),
                              C.c_void_p(cnt.data_ptr()), 1, C.c_void_p(s)), "rt_trace_rays")
    torch.cuda.synchronize()
    c = [int(x) for x in cnt.tolist()]
    times = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        check(lib().rt_trace_rays(ds.handle, C.c_void_p(rays.data_ptr()), n, C.c_void_p(hits.data_ptr()), None, 0,
                                  C.c_void_p(s)), "rt_trace_rays")
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    ms = float(np.median(times))
    util = (c[1] / 2) / max(1, c[4] * 64)
    return dict(ms=round(ms, 4), Mray_s=round(n / ms / 1e3, 1), ns_per_ray=round(ms * 1e6 / n, 3),
                box_tests_per_ray=round(c[1] / n, 2), prim_tests_per_ray=round(c[2] / n, 2),
                node_iters_per_64_rays=round(c[4] * 64 / n, 2), node_lane_util=round(util, 3),
                leaf_iters_per_64_rays=round(c[5] * 64 / n, 2)), hits.view(n, 2)


results = {}
for spp in (int(x) for x in args.spp.split(",")):
    lib().rt_set_variant(3)
    r = Renderer(cfg.width, cfg.height, state_layout="soa")
    r.render_init()
    buf = torch.empty(2 * args.cap * 4, dtype=torch.float32, device=dev)
    count = torch.zeros(1, dtype=torch.int32, device=dev)
    check(lib().rt_set_ray_dump(C.c_void_p(buf.data_ptr()), args.cap, C.c_void_p(count.data_ptr()), 1), "ray dump")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r.render(ds, spp, cfg.depth, cfg.inputs(), flags=abi.RT_FLAG_COUNT_TESTS)
    e1.record()
    torch.cuda.synchronize()
    lib().rt_set_ray_dump(None, 0, None, 1)
    lib().rt_set_variant(-1)
    frame_rays = int(r.counters[0])
    n = min(int(count.item()), args.cap)
    rays = buf[: 8 * n].view(2 * n, 4)
    o, d = rays[0::2, :3], rays[1::2, :3]
    res = dict(spp=spp, frame_rays=frame_rays, bounce1_rays=n, dump_frame_ms=round(e0.elapsed_time(e1), 3))
    base, hits0 = trace(rays, args.reps)
    res["generation_order"] = base
    orders = {}
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    orders["shuffled"] = torch.randperm(n, device=dev, generator=g)
    octant = ((d[:, 0] < 0).to(torch.int64) | ((d[:, 1] < 0).to(torch.int64) << 1) | ((d[:, 2] < 0).to(torch.int64) << 2))
    orders["octant_then_origin_morton"] = torch.argsort((octant << 30) | morton3(o))
    dn = d / torch.linalg.norm(d, dim=1, keepdim=True).clamp(min=1e-30)
    orders["direction_morton_then_origin"] = torch.argsort((morton3(dn) << 30) | morton3(o))
    # coarse binning (what a one-pass counting sort into buckets would give): octant x an 8x8x8 grid of origin cells,
    # generation order kept inside a bucket
    cell = morton3(o) >> 21  # top 3 bits per axis of the 10-bit Morton code
    orders["octant_origin_cell8_binned"] = torch.argsort((octant << 9) | cell, stable=True)
    # the full sort restricted to chunks of 4 Mi rays in generation order (a wavefront whose ray state stays in the
    # 256 MB Infinity Cache: 4 Mi rays x 64 B)
    key = (octant << 30) | morton3(o)
    chunk = 1 << 22
    cp = torch.empty(n, dtype=torch.int64, device=dev)
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        cp[c0:c1] = c0 + torch.argsort(key[c0:c1])
    orders["octant_then_origin_morton_in_4Mi_chunks"] = cp
    del key
    pairs = rays.view(n, 8)
    for name, perm in orders.items():
        pr = pairs[perm].contiguous().view(2 * n, 4)  # one gather into a fresh contiguous buffer
        chk = torch.randint(0, n, (4096,), device=dev)
        assert torch.equal(pr.view(n, 8)[chk], pairs[perm[chk]]), name
        m, h = trace(pr, args.reps)
        back = torch.empty_like(h)
        back[perm] = h
        m["same_hits_as_generation_order"] = bool(torch.equal(back, hits0))
        m["speedup_vs_generation_order"] = round(base["ms"] / m["ms"], 3)
        res[name] = m
        del pr
    results[f"spp{spp}"] = res
    print(json.dumps(res), flush=True)
    del buf, rays

os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
with open(args.out, "w") as f:
    json.dump(results, f, indent=1)
