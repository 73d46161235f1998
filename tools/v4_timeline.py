"""Where a persistent-kernel (v4, or with --variant 6 the persistent flat kernel) frame's time goes: C5 (1 spp, depth 4/1) and C2 at 1 spp.

For each case the frame is rendered with the v4 wave trace (rt_set_wave_trace: per persistent wave its start, the
moment its work queue ran dry, its end and the pixels it took, s_memrealtime at 100 MHz) and timed with HIP events
around the launch (rt_set_timing: queue-head reset + kernel).  The frame splits into
  launch   = event time - device span (queue reset, dispatch of the first wave, end-of-kernel drain);
  ramp     = first wave start -> last wave start (the dispatcher filling the device);
  steady   = last wave start -> first wave whose queue ran dry;
  tail     = first dry queue -> last wave end (waves finishing their last pixels while others are idle).
Then the same frame under the queue knobs (RT_TUNE_QUEUE_CHUNK / _STRIDE) and grid sizes (RT_TUNE_PERSISTENT_WAVES).
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
ap.add_argument("--frames", type=int, default=12)
ap.add_argument("--sweep", action="store_true")
ap.add_argument("--detail", action="store_true", help="per-wave percentiles of the dry and end times")
ap.add_argument("--cases", type=int, default=0, help="only the first N cases (0: all)")
ap.add_argument("--variant", type=int, default=4, help="persistent kernel: 4 (v4, BVH) or 6 (persistent flat)")
args = ap.parse_args()

c5 = scenes.CONFIGS["c5"]
ds5 = DeviceScene(c5.scene_desc())
ds2 = DeviceScene(scenes.builtin(scenes.CONFIGS["c2"].scene))
trace = torch.zeros(8 * 65536, dtype=torch.int64, device="cuda")  # 8 words per wave (kWaveTraceWords)


def run(ds, cfg, spp, depth, flags, rng="xorwow", layout="soa", n=None, traced=True):
    n = n or args.frames
    lib().rt_set_variant(args.variant)
    r = Renderer(cfg.width, cfg.height, rng=rng, state_layout=layout)
    r.render_init()
    times, spans = [], []
    lib().rt_set_timing(1)
    for f in range(n):
        pos, fwd = scenes.moving_camera(f, 60)
        inp = scenes.camera_inputs(pos, fwd, cfg.fov) if cfg is c5 else cfg.inputs()
        if r.accum is not None:
            r.reset_accumulation()
        trace.zero_()
        lib().rt_set_wave_trace(trace.data_ptr() if traced else None, trace.numel())
        r.render(ds, spp, depth, inp, flags=flags)
        torch.cuda.synchronize()
        lib().rt_set_wave_trace(None, 0)
        times.append(lib().rt_last_kernel_ms())
        t = trace.cpu().numpy().reshape(-1, 8)
        t = t[t[:, 0] > 0].astype(np.float64)
        if traced and len(t):
            spans.append(t)
    lib().rt_set_timing(0)
    lib().rt_set_variant(-1)
    ms = float(np.median(times))
    if not spans:
        return ms, None
    t = spans[len(spans) // 2]
    t0 = t[:, 0].min()
    start, dry, end, px = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0, (t[:, 2] - t0) / 100.0, t[:, 3]
    dry = np.where(t[:, 1] > 0, dry, end)
    span = end.max()
    d = dict(ms=ms, waves=len(t), span_us=span, launch_us=ms * 1e3 - span, ramp_us=start.max(),
             ramp90_us=np.percentile(start, 90), steady_us=dry.min() - start.max(), tail_us=span - dry.min(),
             px_median=np.median(px), px_p10=np.percentile(px, 10), px_p90=np.percentile(px, 90),
             life_median_us=np.median(end - start), dry_pct=np.percentile(dry, [10, 50, 90, 99]),
             end_pct=np.percentile(end, [10, 50, 90, 99]))
    return ms, d


def show(name, res):
    ms, d = res
    if d is None:
        print(f"{name:52s} {ms:.3f} ms", flush=True)
        return
    print(f"{name:52s} {ms:.3f} ms | waves {d['waves']} | launch {d['launch_us']:.1f} us, ramp {d['ramp_us']:.1f} "
          f"(p90 {d['ramp90_us']:.1f}), steady {d['steady_us']:.1f}, tail {d['tail_us']:.1f} (span {d['span_us']:.1f}) | "
          f"pixels/wave p10/50/90 {d['px_p10']:.0f}/{d['px_median']:.0f}/{d['px_p90']:.0f}, wave life "
          f"{d['life_median_us']:.1f} us", flush=True)
    if args.detail:
        f = lambda a: "/".join(f"{v:.0f}" for v in a)
        print(f"{'':52s} wave dry p10/50/90/99 {f(d['dry_pct'])} us, wave end p10/50/90/99 {f(d['end_pct'])} us",
              flush=True)


acc = abi.RT_FLAG_ACCUMULATE
cases = [("c5 1 spp depth 4 (as configured)", dict(ds=ds5, cfg=c5, spp=1, depth=4, flags=acc)),
         ("c5 depth 1", dict(ds=ds5, cfg=c5, spp=1, depth=1, flags=acc)),
         ("c5 depth 4, no accumulation", dict(ds=ds5, cfg=c5, spp=1, depth=4, flags=0)),
         ("c5 depth 4, philox (no state)", dict(ds=ds5, cfg=c5, spp=1, depth=4, flags=acc, rng="philox")),
         ("c5 depth 1, philox, no accumulation", dict(ds=ds5, cfg=c5, spp=1, depth=1, flags=0, rng="philox")),
         ("c2 scene 1 spp depth 8", dict(ds=ds2, cfg=scenes.CONFIGS["c2"], spp=1, depth=8, flags=0))]
for name, kw in cases[:args.cases or None]:
    show(name, run(**kw))
    show(name + " [untraced]", run(traced=False, **kw))

if args.sweep:
    for name, base in (("c5", dict(ds=ds5, cfg=c5, spp=1, depth=4, flags=acc)),
                       ("c2 1 spp", dict(ds=ds2, cfg=scenes.CONFIGS["c2"], spp=1, depth=8, flags=0))):
        for chunk in (64, 128, 256, 512, 1024):
            for stride in (128, 4096):
                prev_c = lib().rt_set_tuning(7, chunk)
                prev_s = lib().rt_set_tuning(8, stride)
                show(f"{name} chunk {chunk} stride {stride} B", run(**base))
                lib().rt_set_tuning(7, prev_c)
                lib().rt_set_tuning(8, prev_s)
    for w in (3, 4, 5):
        for chunk in (64, 256):
            prev = lib().rt_set_tuning(2, w)
            prev_c = lib().rt_set_tuning(7, chunk)
            show(f"c5 persistent waves/SIMD {w} chunk {chunk}", run(ds=ds5, cfg=c5, spp=1, depth=4, flags=acc))
            lib().rt_set_tuning(2, prev)
            lib().rt_set_tuning(7, prev_c)
