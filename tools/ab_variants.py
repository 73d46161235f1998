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
ap.add_argument("--thresholds", default="40", help="regen thresholds to try for resumable variants (>= 8)")
ap.add_argument("--leafmax", default="4", help="BVH leaf sizes to try (RT_TUNE_LEAF_MAX)")
ap.add_argument("--pwaves", default="0", help="persistent grid waves/SIMD to try (RT_TUNE_PERSISTENT_WAVES)")
ap.add_argument("--regions", default="2", help="v5 tiles per region to try (RT_TUNE_REGION_TILES; a build with ab_src/v5_region_refill.patch)")
ap.add_argument("--sah", default="16", help="SAH traversal costs x10 to try (RT_TUNE_SAH_TRAVERSAL)")
ap.add_argument("--rng", default="xorwow", choices=("xorwow", "philox"))
args = ap.parse_args()
cfg = scenes.CONFIGS[args.config]
if args.spp:
    cfg = cfg.scaled(cfg.width, cfg.height, args.spp)
variants = []
for sah in (int(x) for x in args.sah.split(",")):
    for lmv in (int(x) for x in args.leafmax.split(",")):
        lm = (lmv, sah)
        for v in (int(v) for v in args.variants.split(",")):
            for th in [int(t) for t in args.thresholds.split(",")]:
                knob = args.pwaves if v == 4 else args.regions if v == 5 else "0"
                for pw in [int(p) for p in knob.split(",")]:
                    variants.append((v, th, lm, pw, 0))
scenes_by_lm = {}
for lm in sorted({v[2] for v in variants}):
    lib().rt_set_tuning(1, lm[0])
    lib().rt_set_tuning(3, lm[1])
    scenes_by_lm[lm] = DeviceScene(scenes.builtin(cfg.scene))
lib().rt_set_tuning(1, 4)
lib().rt_set_tuning(3, 16)
r = Renderer(cfg.width, cfg.height, rng=args.rng)
r.render_init()
inp = cfg.inputs()
times = {v: [] for v in variants}
rays = {}
for v, th, lm, pw, df in variants:  # warm-up / JIT of each variant
    lib().rt_set_variant(v)
    lib().rt_set_tuning(0, th)
    lib().rt_set_tuning(9 if v == 5 else 2, max(pw, 1) if v == 5 else pw)
    r.render(scenes_by_lm[lm], cfg.spp, cfg.depth, inp)
torch.cuda.synchronize()
for rnd in range(args.rounds):
    for v in variants:
        lib().rt_set_variant(v[0])
        lib().rt_set_tuning(0, v[1])
        lib().rt_set_tuning(9 if v[0] == 5 else 2, v[3])
        r.counters.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r.render(scenes_by_lm[v[2]], cfg.spp, cfg.depth, inp)
        e1.record()
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1))
        rays[v] = int(r.counters[0])
for v in variants:
    med = statistics.median(times[v])
    print(f"{args.config} {args.rng} variant {v[0]} thr {v[1]} leafmax {v[2][0]} sah {v[2][1]} {'region' if v[0] == 5 else 'pwaves'} {v[3]}: median {med:.2f} ms  min {min(times[v]):.2f}  {rays[v] / med / 1e6:.3f} Gray/s", flush=True)
