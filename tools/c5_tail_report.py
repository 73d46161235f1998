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
    px = t[:, 3]
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
