"""Headline benchmark: Mray/s of the per-pixel path-trace kernel (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c4] [--variant -1] [--tiled-devices 0,0]

A step is one frame of the hot path (Kernel.cu:102-158 → librt_hip.so rt_render) over the whole image;
inputs (scene tables, RNG state) are resident in HBM before the timed region.  Rays are counted by the
kernel itself (one closest-hit query = one iteration of color()'s loop, Kernel.cu:39).

  --config c2 (default, the BASELINE metric): N = 1 renders config 2 (1920×1080, 64 spp, depth 8, RTIOW
      final scene).  N > 1 (one process per GPU, launched by torch.distributed.run) is weak scaling: the
      image grows to round(1920·√N) × round(1080·√N) (same camera and field of view, ≈2.07 M pixels per GPU),
      split in block-cyclic 16-row bands, and every step ends with the RCCL gather to rank 0.
  --config c4: BASELINE config 4 as configured, strong scaling: one 7680×4320, 128 spp, depth 8 RTIOW frame
      split over the N ranks in 16-row bands (N = 1 renders all of it) + the RCCL gather, whose time is
      reported apart (gather_ms).
  --tiled-devices d0,d1,…: single process, rt_tiled_* C ABI (one band rank per listed device, peer-copy
      gather): the path a C++ viewer uses without torch.distributed.
"""
from __future__ import annotations

import argparse
import re
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
PEAK_HBM_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E ≈ 8 TB/s per GPU
# SURVEY.md §8(d) D4 counted-flop model: AABB test 21, sphere test 23, shading/sky/sampling 60 per ray,
# camera ray 40 per primary sample.
FLOP_BOX, FLOP_PRIM, FLOP_RAY, FLOP_PRIMARY = 21, 23, 60, 40
F_REF_PER_RAY = 21 * 50.7 + 23 * 6.9 + 60  # reference BVH on C2: ≈1.28 kFLOP/ray


def cpu_baseline(cfg: scenes.Config, target_s: float) -> dict:
    """The CPU restatement of the path (oracle/rt_oracle.c built -O3 -march=native -ffp-contract=off on this
    host, OpenMP over rows; it computes the checker's bits, tests/test_oracle.py) on bounded row-strided samples
    of the same frame: on the job's whole CPU share, and on one core."""
    import tempfile

    from oracle import py_oracle as po

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), model)
    except OSError:
        pass
    L = po.native_lib(os.path.join(tempfile.gettempdir(), f"rt_oracle_native_{os.getuid()}"))
    sc = po.OracleScene(scenes.builtin(cfg.scene), library=L)
    inputs = cfg.inputs()
    st = po.init_states(cfg.width, cfg.height)

    def run(first: int, step: int, nthreads: int):
        t0 = time.perf_counter()
        _, _, cnt = po.render(sc, cfg.width, cfg.height, cfg.spp, cfg.depth, inputs, st, rows=(first, cfg.height),
                              row_step=step, threads=nthreads, library=L)
        return cnt.rays, time.perf_counter() - t0, len(range(first, cfg.height, step))

    def sample(first: int, nthreads: int, budget_s: float):
        step = max(1, cfg.height // (2 * nthreads))  # calibration: ~2 rows per thread
        for _ in range(3):  # rescale the row stride until the sample takes about budget_s
            rays, dt, nrows = run(first, step, nthreads)
            if dt >= 0.5 * budget_s or step == 1:
                break
            step = max(1, int(step * dt / budget_s))
        return rays, dt, nrows, step

    rays, dt, nrows, step = sample(1, threads, target_s)
    value = rays / dt / 1e6
    rays1, dt1, nrows1, _ = sample(2, 1, target_s / 3)  # one core: a third of the time budget
    return {"value": round(value, 3), "unit": "Mray/s", "cores": threads, "kind": "port",
            "one_core_Mray_s": round(rays1 / dt1 / 1e6, 3), "host_cpus": os.cpu_count(), "cpu_model": model,
            "build": "gcc -O3 -march=native -ffp-contract=off -fopenmp (oracle/Makefile native), OpenMP over rows",
            "sample": f"rows y = 1, {1 + step}, {1 + 2 * step}, ... ({nrows} of {cfg.height}) of the {cfg.width}x{cfg.height} "
                      f"frame at {cfg.spp} spp, depth {cfg.depth}: {rays} rays in {dt:.2f} s on {threads} threads "
                      f"(the job's CPU share; the host has {os.cpu_count()}); one core: {nrows1} rows, {rays1} rays in "
                      f"{dt1:.2f} s"}


def secondary_mode(cfg: scenes.Config, scene: DeviceScene, inputs, steps: int, rng: str = "philox",
                   state_layout: str = "curand") -> dict:
    """Secondary figure: the same frames with the stateless Philox RNG (RT_FLAG_RNG_PHILOX, no per-pixel
    RNG state in HBM), or with the other XORWOW state layout."""
    r = Renderer(cfg.width, cfg.height, rng=rng, state_layout=state_layout)
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
    state_bytes = 0 if rng == "philox" else (48 if state_layout == "curand" else 24) * cfg.width * cfg.height
    return {"value": round(rays / ms / 1e3, 2), "unit": "Mray/s", "kernel_ms": round(ms, 3),
            "rays_per_frame": int(rays), "hbm_rng_state_bytes": state_bytes}


def pmc_profile(config: str, rng: str, state_layout: str = "curand") -> dict:
    """HBM bytes per launch and SIMD-efficiency counters of the default kernel from the committed rocprofv3
    PMC summary (profiles/pmc_<config>_n1.json, tools/profile_pmc.sh), or {}.  Under weak scaling every
    rank launches the same 1920x1080-sized share, so the N=1 per-launch figures apply per rank."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}_n1.json")
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        d = json.load(f)
    d = d.get("philox", {}) if rng == "philox" else (d.get("soa", {}) if state_layout == "soa" else d)
    keys = ("hbm_bytes_per_launch", "algorithmic_bytes_per_launch", "valu_lane_utilization", "avg_waves_per_simd",
            "ta_busy_frac_per_cu", "kernel")
    return {k: d[k] for k in keys if k in d}


def run_tiled(args, cfg: scenes.Config) -> None:
    """--tiled-devices: one process, rt_tiled_* (band rank r on devices[r], peer-copy gather into one frame)."""
    from cudaraytracer_amd.renderer import TiledRenderer

    devices = [int(d) for d in args.tiled_devices.split(",")]
    lib().rt_set_variant(args.variant)
    t = TiledRenderer(cfg.width, cfg.height, devices, scenes.builtin(cfg.scene), band_rows=16, rng=args.rng)
    inputs = cfg.inputs()
    for _ in range(args.warmup):
        t.render(cfg.spp, cfg.depth, inputs)
    render_ms, gather_ms, rays = [], [], 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        t.render(cfg.spp, cfg.depth, inputs)
        render_ms.append(t.timing.render_ms)
        gather_ms.append(t.timing.gather_ms)
        rays += t.timing.rays
    elapsed = time.perf_counter() - t0
    print(json.dumps({
        "metric": f"Mray/s at {cfg.width}x{cfg.height}, {cfg.spp} spp, depth {cfg.depth}, random-spheres "
                  f"(single-process rt_tiled C-ABI split)",
        "value": round(rays / elapsed / 1e6, 2), "unit": "Mray/s", "n_gpus": len(set(devices)),
        "band_ranks": len(devices), "devices": devices, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32", "rng": args.rng, "data": "synthetic: RTIOW final scene, glibc rand() seed 1",
        "config": {"workload": f"{args.config}: {cfg.width}x{cfg.height}, {cfg.spp} spp, depth {cfg.depth}",
                   "parallelism": f"{len(devices)} band ranks (rt_tiled), 16-row bands, peer-copy gather"},
        "render_ms": round(sum(render_ms) / len(render_ms), 3), "gather_ms": round(sum(gather_ms) / len(gather_ms), 3),
    }), flush=True)
    t.close()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=("c2", "c4"))
    ap.add_argument("--variant", type=int, default=-1, help="kernel variant (rt_set_variant); -1 = automatic")
    ap.add_argument("--rng", choices=("xorwow", "philox"), default="xorwow",
                    help="xorwow: the reference's per-pixel cuRAND state (parity mode, headline); philox: stateless "
                         "Philox4x32-10 streams (RT_FLAG_RNG_PHILOX)")
    ap.add_argument("--state-layout", choices=("soa", "curand"), default="soa",
                    help="XORWOW states: soa = native six uint32 planes (RT_FLAG_STATE_SOA, 24 B/pixel, the same "
                         "streams); curand = the reference's 48-B curandState structs (the LaunchKernel layout)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-philox-line", action="store_true", help="skip the secondary Philox-mode timing (N=1)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank renders on device 0 (use with --backend gloo)")
    ap.add_argument("--tiled-devices", default="",
                    help="single-process multi-device split through the rt_tiled C ABI, e.g. 0,1,2,3 (or 0,0 on one GPU)")
    args = ap.parse_args()

    if args.tiled_devices:
        run_tiled(args, scenes.CONFIGS[args.config])
        return

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
    strong = args.config == "c4"  # one fixed frame split over the ranks
    if world > 1 and not strong:
        s = math.sqrt(world)
        cfg = cfg.scaled(int(round(cfg.width * s)), int(round(cfg.height * s)))
    lib().rt_set_variant(args.variant)

    band = parallel.DEFAULT_BAND_ROWS if world > 1 else cfg.height
    r = Renderer(cfg.width, cfg.height, device=device, band_rows=band, num_ranks=world, rank=rank, rng=args.rng,
                 state_layout=args.state_layout)
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
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
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
        ev[i][2].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = sum(a.elapsed_time(b) for a, b, _ in ev) / args.steps
    gather_ms = sum(b.elapsed_time(g) for _, b, g in ev) / args.steps
    rays = int(r.counters[0].item())
    stats = torch.tensor([elapsed, kernel_ms, gather_ms], dtype=torch.float64, device=red_dev)
    tot = torch.tensor([rays, f_launch], dtype=torch.int64, device=red_dev)
    if world > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    elapsed, kernel_ms, gather_ms = float(stats[0]), float(stats[1]), float(stats[2])
    rays_all = int(tot[0])

    if rank == 0:
        achieved = f_launch / (kernel_ms * 1e-3) / 1e12
        # HBM bytes per launch: the committed N=1 C2 PMC summary.  A rank's bytes do not depend on spp (per pixel:
        # RNG state in and out, one RGBA8 store), so other frame shapes scale it by the rank's pixel count.
        pmc = pmc_profile("c2", args.rng, args.state_layout)
        c2 = scenes.CONFIGS["c2"]
        pix_scale = r.local_rows * cfg.width / (c2.width * c2.height)
        if "hbm_bytes_per_launch" in pmc and pix_scale != 1.0:
            for k in ("hbm_bytes_per_launch", "algorithmic_bytes_per_launch"):
                if k in pmc:
                    pmc[k] = round(pmc[k] * pix_scale)
            pmc["scaled"] = True
        rays_per_launch = c[0]
        hbm_gbps = (round(pmc["hbm_bytes_per_launch"] / (kernel_ms * 1e-3) / 1e9, 2)
                    if "hbm_bytes_per_launch" in pmc else None)
        metric = ("Mray/s (and ms/frame) at 1920x1080, 64 spp, depth 8, random-spheres" if not strong else
                  "Mray/s (and ms/frame) at 7680x4320, 128 spp, depth 8, random-spheres (8-GPU tile-split config)")
        line = {
            "metric": metric,
            "value": round(rays_all / elapsed / 1e6, 2),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "rng": args.rng,
            "state_layout": args.state_layout if args.rng == "xorwow" else None,
            "data": "synthetic: RTIOW final scene (488 spheres) generated from glibc rand() seed 1",
            "config": {
                "workload": (f"{args.config}: {cfg.width}x{cfg.height}, {cfg.spp} spp, depth {cfg.depth}, "
                             + ", ".join(part for part in scenes.CONFIGS[args.config].description.split(", ")
                                         if not re.match(r"\d+ GPUs$|\d+x\d+$|\d+ spp|depth \d+$", part))),
                "width": cfg.width, "height": cfg.height, "spp": cfg.spp, "depth": cfg.depth,
                "parallelism": (f"{world} rank(s) x 16-row bands + {'RCCL' if args.backend == 'nccl' else args.backend} gather"
                                if world > 1 else "1 GPU"),
                "kernel_variant": args.variant,
            },
            "kernel_ms": round(kernel_ms, 3),
            "gather_ms": round(gather_ms, 3) if world > 1 else 0.0,
            "rays_per_frame": rays_all // args.steps,
            "roofline": {
                "bound": "valu",
                "achieved": round(achieved, 3),
                "peak": PEAK_FP32_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                "traffic": pmc.get("hbm_bytes_per_launch"),
                "traffic_source": (("rocprofv3 PMC FETCH_SIZE*2 + WRITE_SIZE, profiles/pmc_c2_n1.json"
                                    + (" (per-pixel bytes x this rank's pixels)" if pmc.get("scaled") else ""))
                                   if "hbm_bytes_per_launch" in pmc else None),
                "algorithmic_hbm_bytes": pmc.get("algorithmic_bytes_per_launch"),
                "hbm_GBps_achieved": hbm_gbps,
                "hbm_frac_of_peak": round(hbm_gbps / PEAK_HBM_GBPS, 5) if hbm_gbps is not None else None,
                "hbm_per_rank": world > 1,
                "simd_lane_utilization": pmc.get("valu_lane_utilization"),
                "waves_per_simd": pmc.get("avg_waves_per_simd"),
                "ta_busy_frac": pmc.get("ta_busy_frac_per_cu"),
                "flop_per_launch": f_launch,
                "flop_per_ray_exec": round(f_launch / max(1, c[0]), 1),
                "flop_per_ray_ref_bvh": round(F_REF_PER_RAY, 1),
                "box_tests_per_ray": round(c[1] / max(1, c[0]), 2),
                "prim_tests_per_ray": round(c[2] / max(1, c[0]), 2),
                "rays_per_launch_rank0": rays_per_launch,
            },
        }
        if world == 1 and args.rng == "xorwow" and not args.no_philox_line and not strong:
            line["philox_mode"] = secondary_mode(cfg, scene, inputs, args.steps)
            other = "curand" if args.state_layout == "soa" else "soa"
            line[f"{other}_state_layout"] = dict(secondary_mode(cfg, scene, inputs, args.steps, "xorwow", other),
                                                 hbm_bytes_per_launch=pmc_profile(args.config, "xorwow", other).get(
                                                     "hbm_bytes_per_launch"))
        if world == 1 and not args.no_cpu_baseline and not strong:
            line["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
