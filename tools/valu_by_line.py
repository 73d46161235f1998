"""Static VALU instruction mix of one kernel per source function and line, from a gfx950 assembly listing compiled
with line tables (`.loc` directives), weighted by the measured issue cost (2 / 4 / 8 cycles per wave64 instruction,
tools/valu_microbench.hip).  Static counts, not executed ones: a branch no lane takes counts as much as
the hot loop — use it to find what the compiler put where (spill reloads, library expansions), then measure.
    hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -mllvm -simplifycfg-sink-common=false \\
        --cuda-device-only -gline-tables-only -S cudaraytracer_amd/csrc/render.hip -o /tmp/render.s
    python tools/valu_by_line.py /tmp/render.s <mangled kernel symbol> [top lines]"""
import bisect
import collections
import os
import re
import sys

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cudaraytracer_amd", "csrc", "render.hip")
FOUR = re.compile(r"v_(cmp|cndmask_b32_e64|min|max|med|lshl|lshr|ashr|mul_u32|mul_lo|mul_hi|mad_u|cvt|bfe|alignbit|"
                  r"readlane|writelane|readfirstlane|mbcnt|perm|ldexp|frexp|div_scale|div_fmas|div_fixup|xad|lshl_add|"
                  r"add3|or3|and_or)")
EIGHT = re.compile(r"v_(sqrt|rcp|rsq|exp|log|sin|cos|pk_)")


def kernel_body(asm_path, symbol):
    out, on = [], False
    for line in open(asm_path):
        if line.startswith(symbol + ":"):
            on = True
        elif on and line.startswith(".Lfunc_end"):
            break
        if on:
            out.append(line.rstrip("\n"))
    if not out:
        sys.exit(f"{symbol} not found in {asm_path}")
    return out


def function_starts(src):
    starts = []
    pat = re.compile(r"^(?:template <.*>\s*)?(?:__device__|__global__|static|inline|constexpr)[^;]*?\b([A-Za-z_]\w*)\s*\(")
    member = re.compile(r"^\s+__device__ [^;]*?\b([A-Za-z_]\w*)\s*\(")
    for i, l in enumerate(src, 1):
        m = pat.match(l) or member.match(l)
        if m and not l.strip().endswith(";"):
            starts.append((i, m.group(1)))
    return sorted(starts)


def main():
    asm, symbol = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    src = open(SRC).read().splitlines()
    starts = function_starts(src)
    keys = [a for a, _ in starts]
    cur = (0, 0)
    by_fn, cyc_fn, by_line = collections.Counter(), collections.Counter(), collections.Counter()
    for l in kernel_body(asm, symbol):
        s = l.strip()
        if s.startswith(".loc"):
            p = s.split()
            cur = (int(p[1]), int(p[2]))
            continue
        if not s.startswith("v_"):
            continue
        w = 8 if EIGHT.match(s) else 4 if FOUR.match(s) else 2
        if cur[0] == 0:
            k = bisect.bisect_right(keys, cur[1]) - 1
            fn = starts[k][1] if k >= 0 else "?"
        else:
            fn = f"(header file {cur[0]})"
        by_fn[fn] += 1
        cyc_fn[fn] += w
        by_line[cur] += 1
    print(f"{'VALU':>6} {'cycles':>7}  function")
    for fn, n in by_fn.most_common(top):
        print(f"{n:6d} {cyc_fn[fn]:7d}  {fn}")
    print(f"{sum(by_fn.values()):6d} {sum(cyc_fn.values()):7d}  total")
    print("\nlines:")
    for (f, ln), n in by_line.most_common(top):
        text = src[ln - 1].strip()[:100] if f == 0 and 0 < ln <= len(src) else ""
        print(f"{n:6d}  {f}:{ln}  {text}")


if __name__ == "__main__":
    main()
