"""Wave lifetime / occupancy timeline of one frame (v3 kernels; rt_set_wave_trace): how long waves live and
how much of the frame is spent in the tail, where fewer waves remain resident than at steady state."""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from cudaraytracer_amd import scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--variant", type=int, default=-1)
ap.add_argument("--warm", action="store_true")
args = ap.parse_args()
cfg = scenes.CONFIGS[args.config]
lib().rt_set_variant(args.variant)
ds = DeviceScene(scenes.builtin(cfg.scene))
r = Renderer(cfg.width, cfg.height)
r.render_init()
waves = ((cfg.width + 7) // 8) * ((cfg.height + 7) // 8)
buf = torch.zeros(2 * waves + 64, dtype=torch.int64, device="cuda")
if args.warm:  # one untraced frame first: the traced frame then runs in the adaptive (longest-first) order
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs())
    torch.cuda.synchronize()
lib().rt_set_wave_trace(buf.data_ptr(), buf.numel())
r.render(ds, cfg.spp, cfg.depth, cfg.inputs())
torch.cuda.synchronize()
lib().rt_set_wave_trace(None, 0)
t = buf[: 2 * waves].cpu().numpy().reshape(-1, 2).astype(np.float64)
t = t[t[:, 0] > 0]
t0 = t[:, 0].min()
s, e = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0  # microseconds
frame = e.max()
life = e - s
grid = np.linspace(0, frame, 201)
resident = np.array([np.sum((s <= g) & (e > g)) for g in grid])
steady = np.median(resident[20:120])
tail_start = grid[np.argmax((grid > frame * 0.3) & (resident < 0.9 * steady))]
print(f"{args.config} variant {args.variant}: {len(t)} waves, frame {frame / 1e3:.2f} ms, wave lifetime "
      f"median {np.median(life) / 1e3:.2f} ms (p10 {np.percentile(life, 10) / 1e3:.2f}, p90 {np.percentile(life, 90) / 1e3:.2f}), "
      f"steady resident waves {steady:.0f} ({steady / 1024:.2f}/SIMD), mean {resident.mean() / 1024:.2f}/SIMD, "
      f"tail (resident < 90% of steady) from {tail_start / 1e3:.2f} ms = {1 - tail_start / frame:.1%} of the frame")
print("resident waves per SIMD at 5% steps:", " ".join(f"{x / 1024:.1f}" for x in resident[::10]))

# Longest-first launch order from this frame's tile lifetimes, then time frames in both orders.
life_by_tile = (buf[: 2 * waves].cpu().numpy().reshape(-1, 2)[:, 1] - buf[: 2 * waves].cpu().numpy().reshape(-1, 2)[:, 0])
order = torch.tensor(np.argsort(-life_by_tile, kind="stable").astype(np.int32), device="cuda")


def timed(n=3):
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r.render(ds, cfg.spp, cfg.depth, cfg.inputs())
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


base = timed()
lib().rt_set_tile_order(order.data_ptr())
ljf = timed()
lib().rt_set_tile_order(None)
base2 = timed()
print(f"frames: {base:.2f} / {base2:.2f} ms (library's adaptive order), host-planned longest-first {ljf:.2f} ms")
