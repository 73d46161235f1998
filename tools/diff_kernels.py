"""Full-frame comparison of two kernel variants (same RNG states in, same scene) and the oracle on the rows where
they differ: which of them follows the reference's arithmetic there.
    python tools/diff_kernels.py --config c3 --a 3 --b 5 [--spp N] [--rng philox]"""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from cudaraytracer_amd import scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer
from oracle import py_oracle as po

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--a", type=int, default=3)
ap.add_argument("--b", type=int, default=5)
ap.add_argument("--spp", type=int, default=0)
ap.add_argument("--rows", type=int, default=4, help="differing rows to check against the oracle")
args = ap.parse_args()
cfg = scenes.CONFIGS[args.config]
if args.spp:
    cfg = cfg.scaled(cfg.width, cfg.height, args.spp)
sc = scenes.builtin(cfg.scene)
ds = DeviceScene(sc)
out = {}
for v in (args.a, args.b):
    lib().rt_set_variant(v)
    r = Renderer(cfg.width, cfg.height)
    r.render_init()
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs())
    torch.cuda.synchronize()
    out[v] = (r.image().copy(), r.states()[:, :6].copy(), int(r.counters[0]), lib().rt_last_variant())
    del r
ia, sa, ra, va = out[args.a]
ib, sb, rb, vb = out[args.b]
d = np.argwhere(ia != ib)
ds_ = np.argwhere((sa != sb).any(axis=1))
print(f"{args.config} {cfg.width}x{cfg.height} {cfg.spp} spp: variant {va} rays {ra}, variant {vb} rays {rb}; "
      f"{len(d)} pixels differ, {len(ds_)} RNG states differ", flush=True)
rows = sorted({int(y) for y, _ in d} | {int(i) // cfg.width for i in ds_[:, 0]})[: args.rows]
for y in rows:
    st = po.init_states(cfg.width, cfg.height)
    ref, _, _ = po.render(po.OracleScene(sc), cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st,
                          rows=(y, y + 1), row_step=1, threads=16)
    xs = [int(x) for yy, x in d if yy == y][:8]
    sst = st.reshape(cfg.height, cfg.width, -1)[y, :, :6]
    print(f"row {y}: pixels {xs}: oracle==a {np.array_equal(ref[y], ia[y])} oracle==b {np.array_equal(ref[y], ib[y])}; "
          f"states oracle==a {np.array_equal(sst, sa.reshape(cfg.height, cfg.width, 6)[y])} "
          f"oracle==b {np.array_equal(sst, sb.reshape(cfg.height, cfg.width, 6)[y])}", flush=True)
    for x in xs[:4]:
        print(f"   x {x}: a {ia[y, x]:08x} b {ib[y, x]:08x} oracle {ref[y, x]:08x}", flush=True)
