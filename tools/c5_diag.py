"""Where a C5 frame's time goes: the configured frame against variants with one ingredient removed (round 4 adds
the texel-fetch cases: the same frame with 256x128 images, which stay cache-resident, and with constant albedos).
  python tools/c5_diag.py [--quick]   (--quick: only the configured frame and the texture cases)"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def frames(ds, cfg, flags, variant=-1, layout="curand", rng="xorwow", spp=None, depth=None, n=30):
    lib().rt_set_variant(variant)
    r = Renderer(cfg.width, cfg.height, rng=rng, state_layout=layout)
    r.render_init()
    t = []
    r.counters.zero_()
    for f in range(n):
        pos, fwd = scenes.moving_camera(f, n)
        inp = scenes.camera_inputs(pos, fwd, cfg.fov)
        r.reset_accumulation()
        t.append(timed(lambda: r.render(ds, spp or cfg.spp, depth or cfg.depth, inp, flags=flags)))
    rays = int(r.counters[0]) / n
    return sorted(t)[n // 2], rays


c5 = scenes.CONFIGS["c5"]
ds5 = DeviceScene(c5.scene_desc())
ds2 = DeviceScene(scenes.builtin(scenes.CONFIGS["c2"].scene))
ds5_small = DeviceScene(scenes.builtin(c5.scene, texture_size=(256, 128)))
flat = scenes.builtin(c5.scene, texture_size=(256, 128))
for k in range(len(flat.materials)):
    flat.materials[k].albedo.type, flat.materials[k].albedo.image = abi.RT_CONSTANT, -1
ds5_const = DeviceScene(flat)
acc = abi.RT_FLAG_ACCUMULATE
quick = "--quick" in sys.argv
cases = [("c5 as configured (auto kernel, accumulate, curand states)", dict(ds=ds5, flags=acc)),
         ("  256x128 textures (cache-resident texels)", dict(ds=ds5_small, flags=acc)),
         ("  constant albedos (no texel fetch, no sphere uv)", dict(ds=ds5_const, flags=acc)),
         ("  256x128 textures, philox, no accumulation", dict(ds=ds5_small, flags=0, rng="philox")),
         ("  philox, no accumulation", dict(ds=ds5, flags=0, rng="philox"))]
for name, kw in cases + ([] if quick else [("c5 as configured (v4, accumulate, curand states)", dict(ds=ds5, flags=acc, variant=4)),
                 ("  no accumulation", dict(ds=ds5, flags=0)),
                 ("  plane state layout", dict(ds=ds5, flags=acc, layout="soa")),
                 ("  philox (no state)", dict(ds=ds5, flags=acc, rng="philox")),
                 ("  v3 kernel", dict(ds=ds5, flags=acc, variant=3)),
                 ("  depth 1", dict(ds=ds5, flags=acc, depth=1)),
                 ("  4 spp", dict(ds=ds5, flags=acc, spp=4)),
                 ("  RTIOW scene (no textures) 1 spp depth 4", dict(ds=ds2, flags=acc)),
                 ("  RTIOW scene, no accumulation, philox", dict(ds=ds2, flags=0, rng="philox"))]):
    ms, rays = frames(cfg=c5, **kw)
    print(f"{name:55s} {ms:7.3f} ms  {rays / 1e6:6.2f} M rays  {rays / ms / 1e6:6.2f} Gray/s", flush=True)

if quick:
    sys.exit(0)
# host-side cost of one rt_render call (no synchronisation inside) and the kernel's own time (HIP events
# recorded by librt_hip.so right around the launch, rt_set_timing)
import time
lib().rt_set_variant(-1)
r = Renderer(c5.width, c5.height)
r.render_init()
inp = c5.inputs()
r.render(ds5, c5.spp, c5.depth, inp, flags=acc)
torch.cuda.synchronize()
host = []
for _ in range(20):
    t0 = time.perf_counter()
    r.render(ds5, c5.spp, c5.depth, inp, flags=acc)
    host.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize()
lib().rt_set_timing(1)
kern = []
for _ in range(20):
    r.render(ds5, c5.spp, c5.depth, inp, flags=acc)
    torch.cuda.synchronize()
    kern.append(lib().rt_last_kernel_ms())
lib().rt_set_timing(0)
host.sort(); kern.sort()
print(f"rt_render host time per call (python -> return): median {host[10]:.3f} ms; kernel (events around the launch): median {kern[10]:.3f} ms")
t0 = time.perf_counter()
for _ in range(50):
    r.render(ds5, c5.spp, c5.depth, inp, flags=acc)
torch.cuda.synchronize()
print(f"50 frames back to back: {(time.perf_counter() - t0) * 1e3 / 50:.3f} ms per frame")
