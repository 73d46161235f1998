"""Interleaved A/B timing of kernel variants on one config (one process, rounds interleaved)."""
import argparse, os, statistics, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cudaraytracer_amd import scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--variants", default="1,6,7")
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--spp", type=int, default=0)
args = ap.parse_args()
cfg = scenes.CONFIGS[args.config]
if args.spp:
    cfg = cfg.scaled(cfg.width, cfg.height, args.spp)
variants = [int(v) for v in args.variants.split(",")]
ds = DeviceScene(scenes.builtin(cfg.scene))
r = Renderer(cfg.width, cfg.height)
r.render_init()
inp = cfg.inputs()
times = {v: [] for v in variants}
rays = {}
for v in variants:  # warm-up / JIT of each variant
    lib().rt_set_variant(v)
    r.render(ds, cfg.spp, cfg.depth, inp)
torch.cuda.synchronize()
for rnd in range(args.rounds):
    for v in variants:
        lib().rt_set_variant(v)
        r.counters.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r.render(ds, cfg.spp, cfg.depth, inp)
        e1.record()
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1))
        rays[v] = int(r.counters[0])
for v in variants:
    med = statistics.median(times[v])
    print(f"{args.config} variant {v}: median {med:.2f} ms  min {min(times[v]):.2f}  {rays[v] / med / 1e6:.3f} Gray/s", flush=True)
