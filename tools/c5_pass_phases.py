"""Offline: the persistent flat kernel's sampled passes (tools/c5_tail.py pass records) binned by start time — the
median / p90 duration of each phase (trace, shade, queue) and the lanes busy — to see whether a C5 frame's tail is
made of slow passes or of late pixels.   python tools/c5_pass_phases.py gpurun_out/c5_tail/<case>.npz [...]"""
import sys

import numpy as np

M = (1 << 40) - 1
for path in sys.argv[1:]:
    z = np.load(path)
    tr, ps, ms = z["trace"].astype(np.int64), z["passes"].astype(np.int64), z["ms"]
    k = int(np.argsort(ms)[len(ms) // 2])
    p, t = ps[k], tr[k]
    t0 = (t[t[:, 0] > 0, 0] & M).min()
    ends = np.sort(((t[t[:, 0] > 0, 2] & M) - t0) * 0.01)
    rows = []
    for w in range(p.shape[0]):
        rec = p[w].reshape(-1, 4)
        rec = rec[rec[:, 0] > 0]
        st, a, b, c = (((rec[:, j] & M) - t0) * 0.01 for j in range(4))
        na = (rec[:, 0] >> 54) & 127
        rows += [(st[i], a[i] - st[i], b[i] - a[i], c[i] - b[i], na[i]) for i in range(len(rec))]
    rows = np.array(rows)
    print(f"{path}: frame {np.median(ms):.3f} ms, {len(rows)} sampled passes, wave end p10/50/90/max "
          f"{np.percentile(ends, [10, 50, 90, 100]).round(0).tolist()} us")
    for lo, hi in [(0, 50), (50, 100), (100, 150), (150, 175), (175, 200), (200, 225), (225, 400)]:
        m = (rows[:, 0] >= lo) & (rows[:, 0] < hi)
        if m.sum():
            r = rows[m]
            q = lambda j: f"{np.median(r[:, j]):5.1f}/{np.percentile(r[:, j], 90):5.1f}"
            print(f"  start {lo:3d}-{hi:3d} us: {m.sum():4d} passes, trace {q(1)} shade {q(2)} queue {q(3)} us "
                  f"(median/p90), lanes busy {np.median(r[:, 4]):.0f}")
