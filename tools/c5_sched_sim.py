"""C5: pass-level simulation of the persistent kernel's schedules on measured per-pixel pass counts.

Input: gpurun_out/c5_cost.npz (tools/c5_cost_dump.py): per work index the loop passes its pixel took on the GPU.
Model: every resident wave runs its passes in lock step (one pass = one time unit, ~9 us on C5); a lane's pixel of
cost c occupies c passes, and the lane takes its next pixel at the end of the last one (the kernel takes and starts a
pixel in the same pass).  What differs between schedules is only which lane gets which work index when — so the
simulation measures the frame's length in passes, the steady phase (until the queue runs dry) and the tail, and the
lanes idle, for:

  wave   : today's kernel — 4096 one-wave workgroups, 16 queue heads (wave w starts on head w % 16, moves to the next
           live head when its own is exhausted), chunks of 128 while the head had > 4 chunks left at the wave's last
           grab, else 64; the next chunk taken when <= 32 indices are left (prefetch); every lane that starts a pixel
           also reserves its NEXT pixel while its head holds > 1/8 of its range (the state prefetch).
  group  : 256 workgroups of 16 waves (one per CU), each owning a static interleaved share of the frame's 8x8 tiles
           (tile k of the frame to group k % 256) handed to its lanes through an LDS counter (no reserve beyond what
           lanes hold), then a global queue over the last FRAC of the tiles in chunks of CHUNK indices; the next-pixel
           reservation while the group's own share has > NEXT_STOP indices left.

  python tools/c5_sched_sim.py [--frames 0,1,2,3] [--frac 0.1] [--chunk 64] [--next-stop 2048]
"""
import argparse

import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("--npz", default="gpurun_out/c5_cost.npz")
ap.add_argument("--frames", default="0")
ap.add_argument("--frac", type=float, default=0.1)
ap.add_argument("--chunk", type=int, default=64)
ap.add_argument("--next-stop", type=int, default=2048)
ap.add_argument("--seed", type=int, default=1)
ap.add_argument("--wave-chunk", action="store_true", help="group: the global queue's chunks per wave, not per group")
args = ap.parse_args()

data = np.load(args.npz)
W_WAVES, HEADS = 4096, 16


def run(cost, policy, rng):
    n = cost.size
    tiles = n // 64
    cur = np.zeros((W_WAVES, 64), np.int32)     # passes left of the lane's pixel (0: needs one)
    nxt = np.full((W_WAVES, 64), -1, np.int32)  # reserved next pixel's cost (-1: none)
    alive = np.ones(W_WAVES, bool)
    end = np.zeros(W_WAVES, np.int32)
    busy = []
    if policy == "wave":
        per = (tiles + HEADS - 1) // HEADS * 64
        head = np.zeros(HEADS, np.int64)         # indices taken per head
        qc = np.arange(W_WAVES) % HEADS
        wq = np.zeros((W_WAVES, 2), np.int64)    # chunk [next, end)
        hl = np.full(W_WAVES, 1 << 40, np.int64)  # head_left at last grab
        dry = np.zeros(W_WAVES, bool)

        def grab(w):
            while True:
                h = qc[w]
                want = 128 if hl[w] > 4 * 128 else 64
                base = head[h]
                lim = min(per, n - h * per)
                if base >= lim:
                    live = [k for k in range(HEADS) if head[k] < min(per, n - k * per)]
                    if not live:
                        dry[w] = True
                        return False
                    above = [k for k in live if k > h]
                    qc[w] = above[0] if above else live[0]
                    hl[w] = 0
                    continue
                take = min(want, lim - base)
                head[h] += take
                wq[w] = (h * per + base, h * per + base + take)
                hl[w] = lim - base - take
                return True

        def take(w, k):  # k indices for wave w (fewer if the queue is dry)
            got = []
            while len(got) < k and not dry[w]:
                if wq[w, 0] >= wq[w, 1] and not grab(w):
                    break
                m = min(k - len(got), wq[w, 1] - wq[w, 0])
                got.extend(range(wq[w, 0], wq[w, 0] + m))
                wq[w, 0] += m
            return got

        def next_ok(w):
            return hl[w] > per // 8
    else:
        G = 256
        WPG = W_WAVES // G
        static_tiles = int(round(tiles * (1.0 - args.frac)))
        own = [np.arange(g, static_tiles, G) for g in range(G)]
        own_next = np.zeros(G, np.int64)         # indices of the group's share handed out
        gq = [static_tiles * 64]                 # the global queue's next index
        gchunk = np.zeros((W_WAVES if args.wave_chunk else G, 2), np.int64)
        dry = np.zeros(W_WAVES, bool)

        def take(w, k):
            g = w // WPG
            got = []
            left = own[g].size * 64 - own_next[g]
            m = int(min(k, left))
            for j in range(own_next[g], own_next[g] + m):
                got.append(int(own[g][j // 64]) * 64 + j % 64)
            own_next[g] += m
            c = w if args.wave_chunk else g
            while len(got) < k:
                if gchunk[c, 0] >= gchunk[c, 1]:
                    if gq[0] >= n:
                        dry[w] = True
                        break
                    b = gq[0]
                    e = min(n, b + args.chunk)
                    gq[0] = e
                    gchunk[c] = (b, e)
                m = int(min(k - len(got), gchunk[c, 1] - gchunk[c, 0]))
                got.extend(range(gchunk[c, 0], gchunk[c, 0] + m))
                gchunk[c, 0] += m
            return got

        def next_ok(w):
            g = w // WPG
            return own[g].size * 64 - own_next[g] > args.next_stop

    t = 0
    first_dry = None
    order = np.arange(W_WAVES)
    while alive.any():
        t += 1
        rng.shuffle(order)
        for w in order:
            if not alive[w]:
                continue
            need = np.nonzero(cur[w] == 0)[0]
            if need.size:
                started = []
                for l in need:
                    if nxt[w, l] >= 0:
                        cur[w, l] = nxt[w, l]
                        nxt[w, l] = -1
                        started.append(l)
                rest = [l for l in need if cur[w, l] == 0]
                got = take(w, len(rest)) if rest else []
                for l, i in zip(rest, got):
                    cur[w, l] = max(1, int(cost[i]))
                    started.append(l)
                if got is not None and len(got) < len(rest) and first_dry is None:
                    first_dry = t
                if next_ok(w):
                    want = [l for l in started if nxt[w, l] < 0]
                    got = take(w, len(want))
                    for l, i in zip(want, got):
                        nxt[w, l] = max(1, int(cost[i]))
            if not (cur[w] > 0).any() and not (nxt[w] >= 0).any() and dry[w]:
                alive[w] = False
                end[w] = t
        busy.append(int((cur > 0).sum()))
        cur = np.maximum(cur - 1, 0)
    return t, first_dry, end, np.array(busy)


frames = [int(f) for f in args.frames.split(",")]
for f in frames:
    cost = data["cost"][f].astype(np.int32)
    for policy in ("wave", "group"):
        T, fd, end, busy = run(cost, policy, np.random.default_rng(args.seed))
        lanes = W_WAVES * 64
        print(f"frame {f} {policy:5s}: {T} passes, first dry {fd}, tail {T - (fd or T)}; wave end p10/50/90/99 "
              f"{np.percentile(end, [10, 50, 90, 99]).round(1).tolist()}; lane-passes busy {busy.sum() / (T * lanes):.3f}",
              flush=True)
