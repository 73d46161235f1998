"""Class the pixels where the reference's BVH closest hit and the geometric closest hit disagree (C4 whole frame, v3).

v3 returns the geometric closest hit; the reference's BVHNode::Hit (Hittable.cuh:387-439) can return another answer
when two primitives tie at the same t or when a box's slab test rejects a ray at its precision edge.  This compiles the
oracle with -DORC_HIT_DIAG into /tmp (never the tests' library), renders the given rows of a config in reference-BVH
mode and prints, per row, the cumulative disagreements: [total, tie, culled, other] (oracle/rt_oracle.c world_hit).

  python tools/bvh_hit_class.py --config c4 --rows 936,1000,1509,1510,1761,2024
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cudaraytracer_amd import scenes
from oracle import py_oracle as po

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c4")
ap.add_argument("--rows", default="936,1000,1509,1510,1761,2024")
ap.add_argument("--threads", type=int, default=8)
args = ap.parse_args()

so = "/tmp/liboracle_hit_diag.so"
subprocess.check_call(["gcc", "-O2", "-std=c99", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-shared", "-fopenmp", "-DORC_HIT_DIAG", "-I", ROOT,
                       os.path.join(ROOT, "oracle", "rt_oracle.c"), "-o", so, "-lm"])
L = po._declare(C.CDLL(so))
L.orc_hit_diag.restype, L.orc_hit_diag.argtypes = C.c_ulonglong, [C.c_int]
cfg = scenes.CONFIGS[args.config]
osc = po.OracleScene(scenes.builtin(cfg.scene), library=L)
prev = [0, 0, 0, 0]
for y in (int(v) for v in args.rows.split(",")):
    st = po.init_states(cfg.width, cfg.height)  # the frame's XORWOW states; rows draw only their own pixels' states
    t = time.time()
    _, _, cnt = po.render(osc, cfg.width, cfg.height, cfg.spp, cfg.depth, cfg.inputs(), st, rows=(y, y + 1),
                          threads=args.threads, library=L)
    now = [int(L.orc_hit_diag(k)) for k in range(4)]
    print(json.dumps({"config": args.config, "row": y, "rays": int(cnt.rays),
                      "disagree": now[0] - prev[0], "tie": now[1] - prev[1], "culled": now[2] - prev[2],
                      "other": now[3] - prev[3], "s": round(time.time() - t, 1)}), flush=True)
    prev = now
