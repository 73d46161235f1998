"""Whole-frame parity (not row samples): render a BASELINE config on the GPU with each given kernel variant and the
oracle (its -O3 -march=native build: the same arithmetic, tests/test_oracle.py) over the whole frame, then count the
pixels, RNG states and rays that differ.
    python tools/full_frame_parity.py --config c3 --variants 3,5 [--spp 32] [--rng philox] [--rtl 0]"""
import argparse, json, os, sys, tempfile, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from cudaraytracer_amd import abi, scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer
from oracle import py_oracle as po

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--variants", default="3,5")
ap.add_argument("--spp", type=int, default=0)
ap.add_argument("--rng", default="xorwow", choices=("xorwow", "philox"))
ap.add_argument("--ltr", type=int, default=0, help="1: Random() filled left to right (RT_FLAG_RIUS_LEFT_TO_RIGHT)")
ap.add_argument("--frame", type=int, default=3, help="Philox frame")
args = ap.parse_args()
cfg = scenes.CONFIGS[args.config]
if args.spp:
    cfg = cfg.scaled(cfg.width, cfg.height, args.spp)
philox = args.rng == "philox"
flags = abi.RT_FLAG_RIUS_LEFT_TO_RIGHT if args.ltr else 0
sc = scenes.builtin(cfg.scene)
inputs = cfg.inputs() if args.config != "c5" else scenes.camera_inputs(*scenes.moving_camera(0, 60), cfg.fov)
L = po.native_lib(os.path.join(tempfile.gettempdir(), f"rt_oracle_native_{os.getuid()}"))
threads = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
t0 = time.time()
st = None if philox else po.init_states(cfg.width, cfg.height)
ref, _, cnt = po.render(po.OracleScene(sc, library=L), cfg.width, cfg.height, cfg.spp, cfg.depth, inputs, st,
                        threads=threads, rius_order=0 if args.ltr else 1, philox=philox, seed=1984, frame=args.frame,
                        library=L)
oracle_s = time.time() - t0
ds = DeviceScene(sc)
for v in (int(x) for x in args.variants.split(",")):
    lib().rt_set_variant(v)
    r = Renderer(cfg.width, cfg.height, rng=args.rng)
    r.render_init()
    r.render(ds, cfg.spp, cfg.depth, inputs, flags=flags, frame=args.frame)
    torch.cuda.synchronize()
    img = r.image()
    bad = np.argwhere(img != ref)
    out = {"config": args.config, "width": cfg.width, "height": cfg.height, "spp": cfg.spp, "rng": args.rng,
           "ltr": args.ltr, "variant": v, "ran": lib().rt_last_variant(), "pixels": int(img.size),
           "pixels_differ": int(len(bad)), "rays": int(r.counters[0]), "oracle_rays": int(cnt.rays),
           "oracle_s": round(oracle_s, 1), "first_differ": [[int(y), int(x)] for y, x in bad[:6]]}
    if len(bad):  # how far the differing pixels are off: RGBA8 channel differences (north_star's per-channel tolerance)
        a8 = img[bad[:, 0], bad[:, 1]].view(np.uint8).reshape(-1, 4)[:, :3].astype(np.int32)
        b8 = ref[bad[:, 0], bad[:, 1]].view(np.uint8).reshape(-1, 4)[:, :3].astype(np.int32)
        d = np.abs(a8 - b8)
        out["max_channel_diff"] = int(d.max())
        out["channel_diff_hist"] = {int(k): int(c) for k, c in zip(*np.unique(d.max(axis=1), return_counts=True))}
    if not philox:
        out["states_differ"] = int((r.states()[:, :6] != st[:, :6]).any(axis=1).sum())
    print(json.dumps(out), flush=True)
    del r
lib().rt_set_variant(-1)
