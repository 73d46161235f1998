"""Headline benchmark: Mray/s of the per-pixel path-trace kernel (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5] [--variant -1] [--tiled-devices 0,0]

A step is one frame of the hot path (Kernel.cu:102-158 → librt_hip.so rt_render) over the whole image;
inputs (scene tables, RNG state) are resident in HBM before the timed region.  Rays are counted by the
kernel itself (one closest-hit query = one iteration of color()'s loop, Kernel.cu:39).

  --config c2 (default, the BASELINE metric): N = 1 renders config 2 (1920×1080, 64 spp, depth 8, RTIOW
      final scene).  N > 1 (one process per GPU) is weak scaling: the image grows to round(1920·√N) ×
      round(1080·√N) (same camera and field of view, ≈2.07 M pixels per GPU), split in block-cyclic 16-row
      bands; every frame is gathered to rank 0 over RCCL on the collective's own stream while the next frame
      renders (parallel.BandGather; the last frame's gather is inside the timed region, gather_ms is the part
      of it the render stream waited for).  The line carries other_configs: BASELINE config 4 (the 7680×4320,
      128 spp frame split over the N ranks + RCCL gather) at every N, and configs 5 and 3 at N = 1.
  --config c3: BASELINE config 3 (3840×2160, 256 spp, depth 16, Cornell box), one GPU.
  --config c4: BASELINE config 4 as configured, strong scaling: one 7680×4320, 128 spp, depth 8 RTIOW frame
      split over the N ranks in 16-row bands (N = 1 renders all of it) + the RCCL gather, whose time is
      reported apart (gather_ms).
  --config c5: BASELINE config 5 (1920×1080, 1 spp, depth 4, three 8192×4096 image textures), one GPU: a step
      is one progressive frame of the scripted moving camera (new InputStruct, accumulation reset because the
      camera moved, one RT_FLAG_ACCUMULATE frame).  Roofline against HBM.
  --tiled-devices d0,d1,…: single process, rt_tiled_* C ABI (one band rank per listed device, peer-copy
      gather): the path a C++ viewer uses without torch.distributed.

Multi-GPU launch: under torch.distributed.run (WORLD_SIZE set) every process is one rank on device LOCAL_RANK.
Without a launcher, `--gpus N` (N > 1) starts its own N ranks as a child `torch.distributed.run` before it
touches any GPU, and fails if fewer than N devices are visible (`--share-gpu` rehearses N ranks on device 0).
`--dry-run` exercises that launch path on the CPU: N gloo ranks gather synthetic bands, no GPU and no kernel.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import re
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (importing torch initialises no GPU)
import torch.distributed as dist  # noqa: E402

from cudaraytracer_amd import parallel  # noqa: E402

PEAK_FP32_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 vector (= f32 MFMA) rate
PEAK_HBM_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E ≈ 8 TB/s per GPU
# SURVEY.md §8(d) D4 counted-flop model: AABB test 21, sphere test 23, rectangle test 12, shading/sky/sampling
# 60 per ray, camera ray 40 per primary sample.  The kernel counts sphere and rectangle tests apart
# (RT_FLAG_COUNT_TESTS: counters[2] all primitive tests, counters[16] the rectangle tests among them).
FLOP_BOX, FLOP_SPHERE, FLOP_RECT, FLOP_RAY, FLOP_PRIMARY = 21, 23, 12, 60, 40
F_REF_PER_RAY = 21 * 50.7 + 23 * 6.9 + 60  # reference BVH on C2: ≈1.28 kFLOP/ray
C5_FRAMES = 60  # C5's scripted orbit (scenes.moving_camera)

METRICS = {
    "c2": "Mray/s (and ms/frame) at 1920x1080, 64 spp, depth 8, random-spheres",
    "c3": "Mray/s (and ms/frame) at 3840x2160, 256 spp, depth 16, Cornell-box emissive",
    "c4": "Mray/s (and ms/frame) at 7680x4320, 128 spp, depth 8, random-spheres (8-GPU tile-split config)",
    "c5": "Mray/s (and ms/frame) at 1920x1080, 1 spp progressive, depth 4, textured spheres + moving camera",
}
DATA = {
    "c2": "synthetic: RTIOW final scene (488 spheres) generated from glibc rand() seed 1",
    "c3": "synthetic: Cornell box of 6 rects (5 Lambertian walls + a DiffuseLight) and 2 spheres (glass, "
          "aluminium metal), black background",
    "c4": "synthetic: RTIOW final scene (488 spheres) generated from glibc rand() seed 1",
    "c5": "synthetic: 3 image-textured spheres + ground, three procedural 8192x4096 RGB8 textures "
          "(the reference's asset size; its JPEGs are not decoded here), scripted orbit camera",
}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=("c2", "c3", "c4", "c5"))
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
    ap.add_argument("--no-config-lines", action="store_true",
                    help="N=1 --config c2: skip the BASELINE config 3 and 5 figures attached to the headline line")
    ap.add_argument("--tune", default="",
                    help="rt_set_tuning overrides as key=value[,key=value] (rt_tuning_key in include/rt_hip.h)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the multi-rank launch: N gloo ranks gather synthetic bands (no GPU)")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args) -> int:
    """`--gpus N` without a launcher: start N ranks as a child torch.distributed.run and wait for it.  This
    process touches no GPU (torch.cuda.device_count() does not initialise one on this image)."""
    if not args.dry_run and not args.share_gpu:
        visible = torch.cuda.device_count()
        if visible < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, {visible} visible "
                  f"(use --share-gpu to rehearse {args.gpus} ranks on one device)", file=sys.stderr, flush=True)
            return 2
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.run(cmd, env=env).returncode


def dry_run(args) -> None:
    """The launch path without a GPU: every rank joins a gloo group and gathers a synthetic band buffer of the
    configured frame (its global row indices), and rank 0 checks the reassembled frame; for config 2 the same for
    config 4's frame (the block other_configs.c4 of a GPU run)."""
    from cudaraytracer_amd.renderer import band_rows_of
    from cudaraytracer_amd import scenes

    rank, world, _ = parallel.env_rank()
    if world != args.gpus:
        raise SystemExit(f"bench.py --dry-run: WORLD_SIZE={world} but --gpus {args.gpus}")
    if world > 1:
        parallel.init_process_group("gloo")

    def gather_ok(config: str) -> bool | None:
        cfg = scenes.CONFIGS[config]
        w, h = 64, cfg.height
        rows = band_rows_of(h, parallel.DEFAULT_BAND_ROWS, world, rank)
        local = torch.tensor(rows, dtype=torch.int64).repeat_interleave(w)
        full = parallel.gather_bands(local, w, h, parallel.DEFAULT_BAND_ROWS) if world > 1 else local.view(h, w)
        if rank != 0:
            return None
        return bool(torch.equal(full, torch.arange(h, dtype=torch.int64)[:, None].expand(h, w)))

    ok = gather_ok(args.config)
    oc = {"c4": {"frame_ok": gather_ok("c4"), "height": scenes.CONFIGS["c4"].height, "scaling": "strong",
                 "band_rows": parallel.DEFAULT_BAND_ROWS}} if args.config == "c2" and not args.no_config_lines else None
    if rank == 0:
        line = {"dry_run": True, "world_size": world, "gpus": args.gpus, "config": args.config,
                "band_rows": parallel.DEFAULT_BAND_ROWS, "frame_ok": ok}
        if oc is not None:
            line["other_configs"] = oc
        print(json.dumps(line), flush=True)
        if not ok or (oc is not None and not oc["c4"]["frame_ok"]):
            raise SystemExit("bench.py --dry-run: gathered frame differs")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline(cfg, scene_desc, inputs, target_s: float) -> dict:
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
    sc = po.OracleScene(scene_desc, library=L)
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


def secondary_mode(cfg, scene, inputs, steps: int, rng: str = "philox", state_layout: str = "curand") -> dict:
    """Secondary figure: the same frames with the stateless Philox RNG (RT_FLAG_RNG_PHILOX, no per-pixel
    RNG state in HBM), or with the other XORWOW state layout."""
    from cudaraytracer_amd.renderer import Renderer

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


def run_tiled(args, cfg) -> None:
    """--tiled-devices: one process, rt_tiled_* (band rank r on devices[r], peer-copy gather into one frame)."""
    from cudaraytracer_amd import scenes
    from cudaraytracer_amd._lib import lib
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


def distinct_devices(world: int, device: int) -> int:
    """Number of distinct physical GPUs the ranks render on (by device UUID; ranks may share one with --share-gpu)."""
    try:
        ident = str(torch.cuda.get_device_properties(device).uuid)
    except Exception:  # noqa: BLE001 - older builds: fall back to the ordinal
        ident = f"{socket.gethostname()}:{device}"
    if world == 1:
        return 1
    ids = [None] * world
    dist.all_gather_object(ids, ident)
    return len(set(ids))


def run_rank(args) -> dict | None:
    """One rank's bench of args.config; returns rank 0's JSON line (None elsewhere)."""
    from cudaraytracer_amd import abi, scenes
    from cudaraytracer_amd._lib import lib
    from cudaraytracer_amd.renderer import DeviceScene, Renderer

    rank, world, local_rank = parallel.env_rank()
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU")
    if world > 1 and args.config in ("c3", "c5"):
        raise SystemExit(f"bench.py: --config {args.config} is a one-GPU configuration (BASELINE.json configs 3, 5)")
    device = 0 if args.share_gpu else local_rank
    if world > 1:
        visible = torch.cuda.device_count()
        if device >= visible:
            raise SystemExit(f"bench.py: rank {rank} wants GPU {device}, {visible} visible")
        torch.cuda.set_device(device)
        parallel.init_process_group(args.backend)
    red_dev = torch.device("cpu") if args.backend == "gloo" else torch.device("cuda", device)
    cfg = scenes.CONFIGS[args.config]
    strong = args.config == "c4"  # one fixed frame split over the ranks
    progressive = args.config == "c5"
    if world > 1 and args.config == "c2":
        s = math.sqrt(world)
        cfg = cfg.scaled(int(round(cfg.width * s)), int(round(cfg.height * s)))
    lib().rt_set_variant(args.variant)
    for kv in filter(None, args.tune.split(",")):
        k, v = (int(x) for x in kv.split("="))
        if lib().rt_set_tuning(k, v) < 0:
            raise SystemExit(f"bench.py: rt_set_tuning({k}, {v}) refused")
    n_gpus = distinct_devices(world, device)

    band = parallel.DEFAULT_BAND_ROWS if world > 1 else cfg.height
    r = Renderer(cfg.width, cfg.height, device=device, band_rows=band, num_ranks=world, rank=rank, rng=args.rng,
                 state_layout=args.state_layout)
    scene_desc = cfg.scene_desc()
    scene = DeviceScene(scene_desc)
    inputs = cfg.inputs()
    r.render_init()
    frame_flags = abi.RT_FLAG_ACCUMULATE if progressive else 0

    # Counting pass (untimed, RNG state not advanced): executed box / primitive tests for F_exec.
    r.counters.zero_()
    r.render(scene, cfg.spp, cfg.depth, inputs,
             flags=frame_flags | abi.RT_FLAG_COUNT_TESTS | abi.RT_FLAG_NO_STATE_WRITEBACK)
    torch.cuda.synchronize()
    c = [int(x) for x in r.counters.tolist()]
    f_launch = flop_model(c)

    frame_no = [0]

    def frame_inputs():
        """C5: the next pose of the scripted orbit (the camera moves every frame, so the accumulation restarts)."""
        if not progressive:
            return inputs
        pos, fwd = scenes.moving_camera(frame_no[0] % C5_FRAMES, C5_FRAMES)
        frame_no[0] += 1
        r.reset_accumulation()
        return scenes.camera_inputs(pos, fwd, cfg.fov)

    # multi-rank: frame k's gather runs on the collective's stream while frame k + 1 renders (parallel.BandGather)
    gatherer = parallel.BandGather(cfg.width, cfg.height, band) if world > 1 else None

    def step():
        r.render(scene, cfg.spp, cfg.depth, frame_inputs(), flags=frame_flags)
        if world > 1:
            gatherer.start(r.pos)

    # below 64 spp the library times v3 and v4 on the first frames and then keeps the faster (rt_render's
    # automatic choice): at least 4 untimed frames so the timed ones run the chosen kernel
    warmup = max(args.warmup, 4) if cfg.spp < 64 and args.variant < 0 else args.warmup
    for _ in range(warmup):
        step()
    if world > 1:
        gatherer.finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    r.counters.zero_()
    stream = torch.cuda.current_stream()
    # HIP events on the render stream.  N > 1: three per step (render, then the gather's share of the stream);
    # N = 1: one pair around the K launches — every event record between two launches puts a marker packet between
    # them (~11 us per C5 frame, 4 %, in round 5's ms_per_step), which a viewer's back-to-back frames do not have.
    # kernel_ms is then the stream's time per frame, kernel plus the launch-to-launch gap (rocprofv3 agrees, §4).
    per_step = world > 1
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps if per_step else 1)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    if not per_step:
        ev[0][0].record(stream)
    for i in range(args.steps):
        if per_step:
            ev[i][0].record(stream)
        r.render(scene, cfg.spp, cfg.depth, frame_inputs(), flags=frame_flags)
        if per_step:
            ev[i][1].record(stream)
            gatherer.start(r.pos)  # waits (stream-side) for frame i - 1's gather, then starts frame i's
            ev[i][2].record(stream)
    if not per_step:
        ev[0][1].record(stream)
    if world > 1:
        gatherer.finish()  # the last frame's gather is inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if per_step:
        kernel_ms = sum(a.elapsed_time(b) for a, b, _ in ev) / args.steps
        gather_ms = sum(b.elapsed_time(g) for _, b, g in ev) / args.steps
    else:
        kernel_ms, gather_ms = ev[0][0].elapsed_time(ev[0][1]) / args.steps, 0.0
    rays = int(r.counters[0].item())
    stats = torch.tensor([elapsed, kernel_ms, gather_ms], dtype=torch.float64, device=red_dev)
    tot = torch.tensor([rays, f_launch], dtype=torch.int64, device=red_dev)
    if world > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    elapsed, kernel_ms, gather_ms = float(stats[0]), float(stats[1]), float(stats[2])
    rays_all = int(tot[0])
    gather = None
    if world > 1:  # one more gather of the last frame, alone and synchronous: the transfer's own time
        counts = parallel.local_row_counts(cfg.height, band, world)
        nbytes = (world - 1) * max(counts) * cfg.width * 4  # rank 0 receives every other rank's padded band buffer
        times = []
        for _ in range(3):
            torch.cuda.synchronize()
            dist.barrier()
            g0 = time.perf_counter()
            parallel.gather_bands(r.pos, cfg.width, cfg.height, band, reuse=True)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - g0)
        gs = torch.tensor([min(times)], dtype=torch.float64, device=red_dev)
        dist.all_reduce(gs, op=dist.ReduceOp.MAX)
        gather = {"bytes_to_rank0": nbytes, "sync_ms": round(float(gs[0]) * 1e3, 3),
                  "GBps": round(nbytes / float(gs[0]) / 1e9, 2),
                  "backend": "RCCL (xGMI)" if args.backend == "nccl" else args.backend}

    if rank == 0:
        line = {
            "metric": METRICS[args.config],
            "value": round(rays_all / elapsed / 1e6, 2),
            "unit": "Mray/s",
            "n_gpus": n_gpus,
            "world_size": world,
            "steps": args.steps,
            "warmup": warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "rng": args.rng,
            "state_layout": args.state_layout if args.rng == "xorwow" else None,
            "data": DATA[args.config],
            "config": {
                "workload": (f"{args.config}: {cfg.width}x{cfg.height}, {cfg.spp} spp, depth {cfg.depth}, "
                             + ", ".join(part for part in scenes.CONFIGS[args.config].description.split(", ")
                                         if not re.match(r"\d+ GPUs$|\d+x\d+$|\d+ spp|depth \d+$", part))),
                "width": cfg.width, "height": cfg.height, "spp": cfg.spp, "depth": cfg.depth,
                "parallelism": (f"{world} rank(s) on {n_gpus} GPU(s) x 16-row bands + "
                                f"{'RCCL' if args.backend == 'nccl' else args.backend} gather" if world > 1 else "1 GPU"),
                "kernel_variant": args.variant,
            },
            "kernel_ms": round(kernel_ms, 3),
            "gather_ms": round(gather_ms, 3) if world > 1 else 0.0,
            "rays_per_frame": rays_all // args.steps,
        }
        if gather is not None:
            line["gather"] = gather
        if progressive:
            line["roofline"] = hbm_roofline(args, cfg, r, c, kernel_ms)
        else:
            line["roofline"] = valu_roofline(args, cfg, r, c, f_launch, kernel_ms, world)
        if world == 1 and args.rng == "xorwow" and not args.no_philox_line and args.config in ("c2", "c3"):
            line["philox_mode"] = secondary_mode(cfg, scene, inputs, args.steps)
            if args.config == "c2":
                other = "curand" if args.state_layout == "soa" else "soa"
                line[f"{other}_state_layout"] = dict(secondary_mode(cfg, scene, inputs, args.steps, "xorwow", other),
                                                     hbm_bytes_per_launch=pmc_profile(args.config, "xorwow", other).get(
                                                         "hbm_bytes_per_launch"))
        if world == 1 and not args.no_cpu_baseline and not strong:
            cpu_inputs = inputs if not progressive else scenes.camera_inputs(*scenes.moving_camera(0, C5_FRAMES), cfg.fov)
            line["cpu_baseline"] = cpu_baseline(cfg, scene_desc, cpu_inputs, args.cpu_seconds)
    return line if rank == 0 else None


def flop_model(c) -> int:
    """SURVEY.md §8(d) D4 FLOP per launch from the counting pass's counters (rays, box tests, primitive tests,
    primary samples; [16] = the rectangle tests among the primitive tests)."""
    rects = c[16]
    spheres = c[2] - rects
    return FLOP_BOX * c[1] + FLOP_SPHERE * spheres + FLOP_RECT * rects + FLOP_RAY * c[0] + FLOP_PRIMARY * c[3]


def valu_roofline(args, cfg, r, c, f_launch, kernel_ms, world) -> dict:
    """VALU-bound roofline: counted algorithmic FLOP of rank 0's launch ÷ the kernel
    time (max over ranks), against the FP32 vector peak; HBM bytes from the committed PMC summary."""
    from cudaraytracer_amd import scenes

    achieved = f_launch / (kernel_ms * 1e-3) / 1e12
    # HBM bytes per launch: the committed N=1 PMC summary of this config.  A rank's bytes do not depend on spp
    # (per pixel: RNG state in and out, one RGBA8 store), so other frame shapes scale it by the rank's pixels.
    # (config 4: its own PMC summary when committed, else C2's per-pixel bytes scaled)
    pmc_cfg = args.config if args.config != "c4" or pmc_profile("c4", args.rng, args.state_layout) else "c2"
    pmc = pmc_profile(pmc_cfg, args.rng, args.state_layout)
    base = scenes.CONFIGS[pmc_cfg]
    pix_scale = r.local_rows * cfg.width / (base.width * base.height)
    if "hbm_bytes_per_launch" in pmc and pix_scale != 1.0:
        for k in ("hbm_bytes_per_launch", "algorithmic_bytes_per_launch"):
            if k in pmc:
                pmc[k] = round(pmc[k] * pix_scale)
        pmc["scaled"] = True
    hbm_gbps = round(pmc["hbm_bytes_per_launch"] / (kernel_ms * 1e-3) / 1e9, 2) if "hbm_bytes_per_launch" in pmc else None
    return {
        "bound": "valu",
        "achieved": round(achieved, 3),
        "peak": PEAK_FP32_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
        "scope": ("per rank: rank 0's counted FLOP per launch / the slowest rank's kernel time, against one GPU's "
                  "peak" if world > 1 else "one launch = one frame"),
        "traffic": pmc.get("hbm_bytes_per_launch"),
        "traffic_source": ((f"rocprofv3 PMC FETCH_SIZE*2 + WRITE_SIZE, profiles/pmc_{pmc_cfg}_n1.json"
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
        "sphere_tests_per_ray": round((c[2] - c[16]) / max(1, c[0]), 2),
        "rect_tests_per_ray": round(c[16] / max(1, c[0]), 2),
        "flop_model": f"{FLOP_BOX}/box + {FLOP_SPHERE}/sphere + {FLOP_RECT}/rect + {FLOP_RAY}/ray + "
                      f"{FLOP_PRIMARY}/primary (SURVEY D4)",
        "rays_per_launch_rank0": c[0],
    }


def hbm_roofline(args, cfg, r, c, kernel_ms) -> dict:
    """C5 is the one configuration whose frame moves HBM bytes worth a roofline: per pixel
    the RNG state in and out (24 + 24 B used, either layout; none for Philox), the float4 accumulator written (16 B:
    the scripted camera moves every frame, so every frame restarts the accumulation with RT_FLAG_ACCUMULATE_RESET,
    which writes it without reading it) and the RGBA8 store (4 B).  The texel gathers (3 B per image-texture lookup,
    at most one per ray) are not in the algorithmic figure; the PMC traffic includes them."""
    px = cfg.width * r.local_rows
    per_px = (0 if args.rng == "philox" else 48) + 16 + 4
    algo = per_px * px
    achieved = algo / (kernel_ms * 1e-3) / 1e9
    pmc = pmc_profile("c5", args.rng, args.state_layout)
    return {
        "bound": "hbm",
        "achieved": round(achieved, 2),
        "peak": PEAK_HBM_GBPS,
        "unit": "GB/s",
        "frac": round(achieved / PEAK_HBM_GBPS, 4),
        "traffic": pmc.get("hbm_bytes_per_launch"),
        "traffic_source": "rocprofv3 PMC FETCH_SIZE*2 + WRITE_SIZE, profiles/pmc_c5_n1.json" if pmc else None,
        "algorithmic_hbm_bytes": algo,
        "algorithmic_bytes_per_pixel": per_px,
        "rays_per_launch": c[0],
    }


def other_configs(args, world: int) -> dict | None:
    """BASELINE configs on the same run's clock beside the C2 headline: config 4 (the 7680x4320, 128 spp frame split
    over the N ranks in 16-row bands + the RCCL gather) at every N, configs 5 (the real-time progressive path) and 3
    (Cornell, 256 spp) at N = 1.  Every rank takes part; rank 0 returns the blocks."""
    out = {}
    subs = ([("c5", 20, 3), ("c3", 2, 1)] if world == 1 else []) + [("c4", 2, 1)]
    for name, steps, warmup in subs:
        sub = argparse.Namespace(**vars(args))
        sub.config, sub.steps, sub.warmup = name, steps, warmup
        sub.no_cpu_baseline = sub.no_philox_line = True
        o = run_rank(sub)
        if o is not None:
            out[name] = {k: o[k] for k in ("metric", "value", "unit", "ms_per_step", "kernel_ms", "gather_ms",
                                           "rays_per_frame", "steps", "warmup", "scaling", "roofline") if k in o}
            out[name]["workload"] = o["config"]["workload"]
            out[name]["parallelism"] = o["config"]["parallelism"]
            if "gather" in o:
                out[name]["gather"] = o["gather"]
    return out if parallel.env_rank()[0] == 0 else None


def main() -> None:
    args = parse_args()
    launched = "WORLD_SIZE" in os.environ
    if not launched and args.gpus > 1 and not args.tiled_devices:
        sys.exit(self_launch(args))
    if args.dry_run:
        dry_run(args)
        return
    if args.tiled_devices:
        from cudaraytracer_amd import scenes
        run_tiled(args, scenes.CONFIGS[args.config])
        return
    line = run_rank(args)
    world = parallel.env_rank()[1]
    if args.config == "c2" and not args.no_config_lines:
        oc = other_configs(args, world)
        if line is not None:
            line["other_configs"] = oc
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if line is not None:
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
