"""C5's tail, per XCD and per CU: render C5 frames on the persistent flat kernel (variant 6) with
the 8-word wave trace (rt_set_wave_trace: start, queue dry, end, pixels, HW_ID | XCC_ID << 32, last pixel handed
out, chunk grabs | exhausted-head probes << 32, ticks waiting for queue atomics) and save the raw traces, one .npz
per case, for offline analysis (tools/c5_tail_report.py).

  python tools/c5_tail.py --out gpurun_out/c5_tail  [--frames 6] [--variant 6]
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

WORDS = 8  # kWaveTraceWords (render.hip)
PASS_WORDS = 1024  # kPassTrace: per-pass stamps of every 64th wave (persistent flat kernel)

ap = argparse.ArgumentParser()
ap.add_argument("--out", default="gpurun_out/c5_tail")
ap.add_argument("--frames", type=int, default=6)
ap.add_argument("--variant", type=int, default=6)
ap.add_argument("--tune", default="", help="k=v,...[;k=v,...] rt_set_tuning sets: every case runs under each set")
ap.add_argument("--cases", default="d4,d1,d1p")
args = ap.parse_args()
os.makedirs(args.out, exist_ok=True)

c5 = scenes.CONFIGS["c5"]
ds5 = DeviceScene(c5.scene_desc())
trace = torch.zeros(WORDS * 65536, dtype=torch.int64, device="cuda")
ACC = abi.RT_FLAG_ACCUMULATE
CASES = {"d4": dict(depth=4, flags=ACC, rng="xorwow"),   # as configured
         "d1": dict(depth=1, flags=ACC, rng="xorwow"),   # one trace + one shade per pixel
         "d1p": dict(depth=1, flags=0, rng="philox")}    # no state, no accumulator


def run(name, depth, flags, rng, tag=""):
    lib().rt_set_variant(args.variant)
    r = Renderer(c5.width, c5.height, rng=rng, state_layout="soa")
    r.render_init()
    lib().rt_set_timing(1)
    ms, traces, passes = [], [], []
    for f in range(args.frames + 2):
        pos, fwd = scenes.moving_camera(f, 60)
        inp = scenes.camera_inputs(pos, fwd, c5.fov)
        r.reset_accumulation()
        traced = f >= 2
        trace.zero_()
        lib().rt_set_wave_trace(trace.data_ptr() if traced else None, trace.numel())
        r.render(ds5, c5.spp, depth, inp, flags=flags)
        torch.cuda.synchronize()
        lib().rt_set_wave_trace(None, 0)
        if traced:
            ms.append(lib().rt_last_kernel_ms())
            full = trace.cpu().numpy()
            grid = int(full[3]) >> 32  # (wave 0's record: pixels | grid << 32)
            t = full[:WORDS * grid].reshape(-1, WORDS)
            traces.append(t[t[:, 0] > 0].copy())
            passes.append(full[WORDS * grid:WORDS * grid + PASS_WORDS * ((grid + 63) // 64)].reshape(-1, PASS_WORDS).copy())
    # untraced frames: the trace's own cost
    plain = []
    for f in range(args.frames):
        pos, fwd = scenes.moving_camera(f, 60)
        r.reset_accumulation()
        r.render(ds5, c5.spp, depth, scenes.camera_inputs(pos, fwd, c5.fov), flags=flags)
        torch.cuda.synchronize()
        plain.append(lib().rt_last_kernel_ms())
    lib().rt_set_timing(0)
    lib().rt_set_variant(-1)
    n = max(len(t) for t in traces)
    arr = np.zeros((len(traces), n, WORDS), np.uint64)
    for i, t in enumerate(traces):
        arr[i, :len(t)] = t.view(np.uint64)
    np.savez_compressed(os.path.join(args.out, f"{name}{tag}.npz"), trace=arr, ms=np.array(ms), plain_ms=np.array(plain),
                        passes=np.stack(passes).view(np.uint64))
    wait = arr[:, :, 7].astype(np.float64).sum(axis=1) * 0.01 / np.maximum(1, (arr[:, :, 0] > 0).sum(axis=1))
    print(f"{name}{tag}: mean atomic wait/wave {np.median(wait):.1f} us, traced {np.median(ms):.3f} ms, untraced {np.median(plain):.3f} ms, waves {n}", flush=True)


for tset in args.tune.split(";"):
    prev = []
    for kv in filter(None, tset.split(",")):
        k, v = (int(x) for x in kv.split("="))
        prev.append((k, lib().rt_set_tuning(k, v)))
    tag = ("_" + tset.replace(",", "_").replace("=", "-")) if tset else ""
    for name in args.cases.split(","):
        run(name, tag=tag, **CASES[name])
    for k, v in reversed(prev):
        lib().rt_set_tuning(k, v)
