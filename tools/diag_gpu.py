"""GPU diagnostic: parity of every kernel variant against the oracle on small configs + C2 timing."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, ctypes as C
from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd.renderer import Renderer, DeviceScene
from cudaraytracer_amd._lib import lib
from oracle import py_oracle as po

def compare(a, b):
    ab = a.view(np.uint8).reshape(-1, 4)[:, :3].astype(np.int32)
    bb = b.view(np.uint8).reshape(-1, 4)[:, :3].astype(np.int32)
    d = np.abs(ab - bb)
    px_exact = np.mean(np.all(d == 0, axis=1))
    return dict(exact=float(px_exact), within1=float(np.mean(np.all(d <= 1, axis=1))), maxdiff=int(d.max()), mean=float(d.mean()))

cases = [("c1", scenes.CONFIGS["c1"]), ("rtiow", scenes.CONFIGS["c2"].scaled(192, 112, 16)),
         ("cornell", scenes.CONFIGS["c3"].scaled(128, 128, 16)), ("default", scenes.CONFIGS["default"].scaled(160, 120, 8)),
         ("textured", scenes.CONFIGS["c5"].scaled(160, 96, 4))]
variants = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 1, 2, 3, 4, 5]
for name, cfg in cases:
    sc = scenes.builtin(cfg.scene)
    osc = po.OracleScene(sc)
    inp = cfg.inputs()
    st = po.init_states(cfg.width, cfg.height)
    t = time.time()
    ref, _, cnt = po.render(osc, cfg.width, cfg.height, cfg.spp, cfg.depth, inp, st, threads=16)
    ot = time.time() - t
    ds = DeviceScene(sc)
    print(f"{name}: oracle {ot:.2f}s rays {cnt.rays} nodes {ds.info().num_nodes} depth {ds.info().bvh_depth}", flush=True)
    for v in variants:
        lib().rt_set_variant(v)
        r = Renderer(cfg.width, cfg.height)
        r.render_init()
        r.counters.zero_()
        try:
            r.render(ds, cfg.spp, cfg.depth, inp)
            torch.cuda.synchronize()
        except Exception as e:
            print(f"  variant {v}: {e}"); continue
        img = r.image()
        stc = r.states()
        print(f"  variant {v}: {compare(img, ref)} rays {int(r.counters[0])} state_eq {bool(np.array_equal(stc[:, :6], st[:, :6]))}", flush=True)

cfg = scenes.CONFIGS["c2"]
sc = scenes.builtin(cfg.scene)
ds = DeviceScene(sc)
inp = cfg.inputs()
r = Renderer(cfg.width, cfg.height)
r.render_init()
for v in variants:
    lib().rt_set_variant(v)
    for it in range(3):
        r.counters.zero_()
        torch.cuda.synchronize()
        t = time.time()
        r.render(ds, cfg.spp, cfg.depth, inp)
        torch.cuda.synchronize()
        dt = time.time() - t
        rays = int(r.counters[0])
        print(f"C2 variant {v} iter {it}: {dt*1e3:.1f} ms  rays {rays}  {rays/dt/1e9:.3f} Gray/s", flush=True)
