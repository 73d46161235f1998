"""Offline report of tools/c5_tail.py's traces (no GPU): where a C5 frame's tail goes, per XCD and per CU.

  python tools/c5_tail_report.py gpurun_out/c5_tail/d1.npz [...]

Per frame (the median frame is shown): the steady phase (last wave start -> first wave that found the queue dry) and
the tail (first dry -> last wave end); per XCD the waves, their start spread, the first and median dry time, the last
end and the time the XCD's waves spent waiting for queue atomics; the waves alive at each point of the tail; and per
wave the gap between its last pixel handed out and its end (one pixel lifetime if the wave ended with its last
pixels)."""
import sys

import numpy as np

TICK_US = 0.01  # s_memrealtime: 100 MHz


def analyse(path):
    z = np.load(path)
    tr, ms = z["trace"].astype(np.int64), z["ms"]
    k = int(np.argsort(ms)[len(ms) // 2])
    t = tr[k]
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    start, dry, end = (t[:, 0] - t0) * TICK_US, (t[:, 1] - t0) * TICK_US, (t[:, 2] - t0) * TICK_US
    dry = np.where(t[:, 1] > 0, dry, end)
    last = np.where(t[:, 5] > 0, (t[:, 5] - t0) * TICK_US, start)
    px = t[:, 3] & 0xFFFFFFFF
    hw = t[:, 4] & 0xFFFFFFFF
    xcc = (t[:, 4] >> 32) & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    grabs, probes = t[:, 6] & 0xFFFFFFFF, t[:, 6] >> 32
    wait = t[:, 7] * TICK_US
    print(f"== {path}: frame {ms[k]:.3f} ms (median of {len(ms)} traced; untraced median {np.median(z['plain_ms']):.3f}),"
          f" {len(t)} waves, span {end.max():.1f} us")
    print(f"   ramp (last start) {start.max():.1f} us, first dry {dry.min():.1f}, steady {dry.min() - start.max():.1f}, "
          f"tail {end.max() - dry.min():.1f} us")
    pc = lambda a: "/".join(f"{v:.0f}" for v in np.percentile(a, [10, 50, 90, 99]))
    print(f"   wave dry p10/50/90/99 {pc(dry)} us; end {pc(end)}; last pixel out {pc(last)}; end - last out {pc(end - last)}")
    print(f"   pixels/wave {pc(px)}; grabs/wave {pc(grabs)}, probes/wave {pc(probes)}; atomic wait/wave {pc(wait)} us "
          f"({wait.sum() / (end - start).sum() * 100:.1f} % of wave time)")
    print("   XCD  waves  start-max  dry-min  dry-p50  end-max  last-out-max  wait-sum(us)  pixels")
    for x in range(8):
        m = xcc == x
        if not m.any():
            continue
        print(f"   {x:3d} {m.sum():6d} {start[m].max():9.1f} {dry[m].min():8.1f} {np.median(dry[m]):8.1f} {end[m].max():8.1f}"
              f" {last[m].max():12.1f} {wait[m].sum():12.0f} {px[m].sum():8d}")
    # waves alive over the tail
    grid = np.linspace(dry.min(), end.max(), 9)
    alive = [int(((start <= g) & (end > g)).sum()) for g in grid]
    print("   waves alive at tail points " + ", ".join(f"{g:.0f}us:{a}" for g, a in zip(grid, alive)))
    # the CUs that finish last
    key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    cu_end = {int(c): end[key == c].max() for c in np.unique(key)}
    slow = sorted(cu_end.items(), key=lambda kv: -kv[1])[:8]
    print("   latest CUs (xcd.se.sh.cu: end us) " + ", ".join(f"{c >> 8}.{(c >> 5) & 7}.{(c >> 4) & 1}.{c & 15}:{e:.0f}"
                                                          for c, e in slow))
    print(f"   CUs seen {len(cu_end)}, CU end p10/50/90 {pc(np.array(list(cu_end.values())))}")


for p in sys.argv[1:]:
    analyse(p)


def passes(path):
    """Per-pass stamps of every 64th wave (persistent flat kernel, 4 words per pass): pass durations split into the
    trace, the shading, the queue and the camera rays, before and after the wave found the queue dry."""
    z = np.load(path)
    if "passes" not in z:
        return
    tr, ms, ps = z["trace"].astype(np.int64), z["ms"], z["passes"].astype(np.int64)
    k = int(np.argsort(ms)[len(ms) // 2])
    t, p = tr[k], ps[k]
    t0 = t[t[:, 0] > 0, 0].min() & 0xFFFFFFFFFF
    rows = {"steady": [], "tail": []}
    npass = []
    for i in range(p.shape[0]):
        w = t[64 * i]
        rec = p[i].reshape(-1, 4)
        rec = rec[rec[:, 0] != 0]
        if len(rec) < 2:
            continue
        st = ((rec[:, 0] & 0xFFFFFFFFFF) - t0) * TICK_US
        a, b, c = ((rec[:, 1] & 0xFFFFFFFFFF) - t0) * TICK_US, ((rec[:, 2] & 0xFFFFFFFFFF) - t0) * TICK_US, \
            ((rec[:, 3] & 0xFFFFFFFFFF) - t0) * TICK_US
        nxt = np.append(st[1:], ((w[2] & 0xFFFFFFFFFF) - t0) * TICK_US)
        act = (rec[:, 0] >> 54) & 0x7F
        dry = (((w[1] if w[1] > 0 else w[2]) & 0xFFFFFFFFFF) - t0) * TICK_US
        for q in range(len(rec)):
            rows["tail" if st[q] >= dry else "steady"].append((nxt[q] - st[q], a[q] - st[q], b[q] - a[q], c[q] - b[q],
                                                               nxt[q] - c[q], act[q]))
        npass.append(len(rec))
    print(f"   sampled waves {len(npass)}, passes/wave p10/50/90 {'/'.join(f'{v:.0f}' for v in np.percentile(npass, [10, 50, 90]))}"
          "; per pass mean us (median): total | trace | shade | queue | camera+loop | lanes with a pixel")
    for name, r in rows.items():
        if not r:
            continue
        r = np.array(r)
        f = lambda j: f"{r[:, j].mean():5.2f} ({np.median(r[:, j]):5.2f})"
        print(f"     {name:6s} {len(r) / max(1, len(npass)):5.1f} passes/wave: {f(0)} | {f(1)} | {f(2)} | {f(3)} | {f(4)} | "
              f"{r[:, 5].mean():.1f}")


for p in sys.argv[1:]:
    passes(p)
