"""Headline benchmark: Mray/s of the per-pixel path-trace kernel (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2] [--variant -1]

A step is one frame of the hot path (Kernel.cu:102-158 → librt_hip.so rt_render) over the whole image;
inputs (scene tables, RNG state) are resident in HBM before the timed region.  N = 1 renders BASELINE
config 2 (1920×1080, 64 spp, depth 8, RTIOW final scene).  N > 1 (one process per GPU, launched by
torch.distributed.run) is weak scaling: the image grows to round(1920·√N) × round(1080·√N) (same camera,
same field of view, ≈2.07 M pixels per GPU), split in block-cyclic 16-row bands, and every step ends with
the RCCL gather of the per-rank framebuffers to rank 0.  Rays are counted by the kernel itself (one
closest-hit query = one iteration of color()'s loop, Kernel.cu:39).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from cudaraytracer_amd import abi, parallel, scenes  # noqa: E402
from cudaraytracer_amd._lib import lib  # noqa: E402
from cudaraytracer_amd.renderer import DeviceScene, Renderer  # noqa: E402

PEAK_FP32_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 vector (= f32 MFMA) rate
# SURVEY.md §8(d) D4 counted-flop model: AABB test 21, sphere test 23, shading/sky/sampling 60 per ray,
# camera ray 40 per primary sample.
FLOP_BOX, FLOP_PRIM, FLOP_RAY, FLOP_PRIMARY = 21, 23, 60, 40
F_REF_PER_RAY = 21 * 50.7 + 23 * 6.9 + 60  # reference BVH on C2: ≈1.28 kFLOP/ray


def cpu_baseline(cfg: scenes.Config, target_s: float) -> dict:
    """The CPU restatement (oracle/, OpenMP) on a bounded, row-strided sample of the same frame."""
    from oracle import py_oracle as po

    threads = min(16, os.cpu_count() or 1)
    sc = po.OracleScene(scenes.builtin(cfg.scene))
    inputs = cfg.inputs()

    def run(step: int):
        st = po.init_states(cfg.width, cfg.height)
        t0 = time.perf_counter()
        _, _, cnt = po.render(sc, cfg.width, cfg.height, cfg.spp, cfg.depth, inputs, st, rows=(0, cfg.height),
                              row_step=step, threads=threads)
        return cnt.rays, time.perf_counter() - t0

    rays, dt = run(max(1, cfg.height // (4 * threads)))  # calibration: 4 rows per thread
    rate = rays / max(dt, 1e-6)
    step = max(1, int(math.ceil(cfg.height * cfg.width * cfg.spp * 3.1 / max(rate * target_s, 1.0))))
    step = min(step, cfg.height)
    rays, dt = run(step)
    nrows = len(range(0, cfg.height, step))
    return {"value": round(rays / dt / 1e6, 3), "unit": "Mray/s", "cores": threads, "kind": "port",
            "sample": f"rows y = 0, {step}, {2 * step}, ... ({nrows} of {cfg.height}) of the {cfg.width}x{cfg.height} "
                      f"frame at {cfg.spp} spp, depth {cfg.depth}: {rays} rays in {dt:.2f} s, {threads} OpenMP threads"}


def philox_mode(cfg: scenes.Config, scene: DeviceScene, inputs, steps: int) -> dict:
    """Secondary figure: the same frames with the stateless Philox RNG (RT_FLAG_RNG_PHILOX, no per-pixel
    RNG state in HBM).  Not the headline: the reference's stream is XORWOW."""
    r = Renderer(cfg.width, cfg.height, rng="philox")
    r.render_init()
    r.render(scene, cfg.spp, cfg.depth, inputs)  # warm-up
    torch.cuda.synchronize()
    r.counters.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        r.render(scene, cfg.spp, cfg.depth, inputs)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    rays = int(r.counters[0]) / steps
    return {"value": round(rays / ms / 1e3, 2), "unit": "Mray/s", "kernel_ms": round(ms, 3),
            "rays_per_frame": int(rays), "hbm_rng_state_bytes": 0}


def pmc_profile(config: str, rng: str) -> dict:
    """HBM bytes per launch and SIMD-efficiency counters of the default kernel from the committed rocprofv3
    PMC summary (profiles/pmc_<config>_n1.json, tools/profile_pmc.sh), or {}.  Under weak scaling every
    rank launches the same 1920x1080-sized share, so the N=1 per-launch figures apply per rank."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}_n1.json")
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        d = json.load(f)
    d = d.get("philox", {}) if rng == "philox" else d
    keys = ("hbm_bytes_per_launch", "algorithmic_bytes_per_launch", "valu_lane_utilization", "avg_waves_per_simd",
            "ta_busy_frac_per_cu", "kernel")
    return {k: d[k] for k in keys if k in d}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--variant", type=int, default=-1, help="kernel variant (rt_set_variant); -1 = automatic")
    ap.add_argument("--rng", choices=("xorwow", "philox"), default="xorwow",
                    help="xorwow: the reference's per-pixel cuRAND state (parity mode, headline); philox: stateless "
                         "Philox4x32-10 streams (RT_FLAG_RNG_PHILOX)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-philox-line", action="store_true", help="skip the secondary Philox-mode timing (N=1)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank renders on device 0 (use with --backend gloo)")
    args = ap.parse_args()

    rank, world, local_rank = parallel.env_rank()
    if world != args.gpus:
        if rank == 0:
            print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}", file=sys.stderr)
    device = 0 if args.share_gpu else local_rank
    if world > 1:
        torch.cuda.set_device(device)
        parallel.init_process_group(args.backend)
    red_dev = torch.device("cpu") if args.backend == "gloo" else torch.device("cuda", device)
    cfg = scenes.CONFIGS[args.config]
    if world > 1:
        s = math.sqrt(world)
        cfg = cfg.scaled(int(round(cfg.width * s)), int(round(cfg.height * s)))
    lib().rt_set_variant(args.variant)

    band = parallel.DEFAULT_BAND_ROWS if world > 1 else cfg.height
    r = Renderer(cfg.width, cfg.height, device=device, band_rows=band, num_ranks=world, rank=rank, rng=args.rng)
    scene = DeviceScene(scenes.builtin(cfg.scene))
    inputs = cfg.inputs()
    r.render_init()

    # Counting pass (untimed, RNG state not advanced): executed box / primitive tests for F_exec.
    r.counters.zero_()
    r.render(scene, cfg.spp, cfg.depth, inputs, flags=abi.RT_FLAG_COUNT_TESTS | abi.RT_FLAG_NO_STATE_WRITEBACK)
    torch.cuda.synchronize()
    c = [int(x) for x in r.counters.tolist()]
    f_launch = FLOP_BOX * c[1] + FLOP_PRIM * c[2] + FLOP_RAY * c[0] + FLOP_PRIMARY * c[3]

    def step():
        r.render(scene, cfg.spp, cfg.depth, inputs)
        if world > 1:
            parallel.gather_bands(r.pos, cfg.width, cfg.height, band)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    r.counters.zero_()
    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        r.render(scene, cfg.spp, cfg.depth, inputs)
        ev[i][1].record(stream)
        if world > 1:
            parallel.gather_bands(r.pos, cfg.width, cfg.height, band)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    rays = int(r.counters[0].item())
    stats = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=red_dev)
    tot = torch.tensor([rays, f_launch], dtype=torch.int64, device=red_dev)
    if world > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    elapsed, kernel_ms = float(stats[0]), float(stats[1])
    rays_all = int(tot[0])

    if rank == 0:
        achieved = f_launch / (kernel_ms * 1e-3) / 1e12
        pmc = pmc_profile(args.config, args.rng) if args.config == "c2" else {}
        rays_per_launch = c[0]
        line = {
            "metric": "Mray/s (and ms/frame) at 1920x1080, 64 spp, depth 8, random-spheres",
            "value": round(rays_all / elapsed / 1e6, 2),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "rng": args.rng,
            "data": "synthetic: RTIOW final scene (488 spheres) generated from glibc rand() seed 1",
            "config": {
                "workload": (f"{args.config}: {cfg.width}x{cfg.height}, {cfg.spp} spp, depth {cfg.depth}, "
                             f"{scenes.CONFIGS[args.config].description.split(', ', 3)[-1]}"),
                "width": cfg.width, "height": cfg.height, "spp": cfg.spp, "depth": cfg.depth,
                "parallelism": f"{world} rank(s) x 16-row bands + gather" if world > 1 else "1 GPU",
                "kernel_variant": args.variant,
            },
            "kernel_ms": round(kernel_ms, 3),
            "rays_per_frame": rays_per_launch,
            "roofline": {
                "bound": "valu",
                "achieved": round(achieved, 3),
                "peak": PEAK_FP32_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                "traffic": pmc.get("hbm_bytes_per_launch"),
                "traffic_source": "rocprofv3 PMC FETCH_SIZE*2 + WRITE_SIZE, profiles/pmc_c2_n1.json" if pmc else None,
                "algorithmic_hbm_bytes": pmc.get("algorithmic_bytes_per_launch"),
                "hbm_GBps_achieved": (round(pmc["hbm_bytes_per_launch"] / (kernel_ms * 1e-3) / 1e9, 2)
                                      if "hbm_bytes_per_launch" in pmc else None),
                "simd_lane_utilization": pmc.get("valu_lane_utilization"),
                "waves_per_simd": pmc.get("avg_waves_per_simd"),
                "ta_busy_frac": pmc.get("ta_busy_frac_per_cu"),
                "flop_per_launch": f_launch,
                "flop_per_ray_exec": round(f_launch / max(1, c[0]), 1),
                "flop_per_ray_ref_bvh": round(F_REF_PER_RAY, 1),
                "box_tests_per_ray": round(c[1] / max(1, c[0]), 2),
                "prim_tests_per_ray": round(c[2] / max(1, c[0]), 2),
            },
        }
        if world == 1 and args.rng == "xorwow" and not args.no_philox_line:
            line["philox_mode"] = philox_mode(cfg, scene, inputs, args.steps)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
