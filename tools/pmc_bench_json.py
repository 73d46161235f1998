"""profiles/pmc_<config>_n1.json (read by bench.py) from tools/profile_pmc.sh runs of one config with the
traffic groups (tools/pmc_groups_traffic.txt), one output directory per RNG mode, last (warm) dispatch of each pass.
    python tools/pmc_bench_json.py [--config c2|c3|c5] <xorwow dir> <philox dir> [<xorwow soa-layout dir>]
        > profiles/pmc_<config>_n1.json

Derived fields (MI355X: 8 XCDs, 256 CUs, 1024 SIMDs; SQ_* counters aggregate over SEs, in quad-cycles):
  hbm_read_bytes_corrected = FETCH_SIZE (KB) x 1024 x 2   (gfx950 reports half of the wide reads,
                                                            /opt/skills/guides/MI355X_MICROARCH.md)
  hbm_write_bytes          = WRITE_SIZE (KB) x 1024
  avg_waves_per_simd       = 4 SQ_WAVE_CYCLES / (1024 x GRBM_GUI_ACTIVE / 8)
  valu_lane_utilization    = SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU)
  ta_busy_frac_per_cu      = TA_TA_BUSY_sum / 256 / (GRBM_GUI_ACTIVE / 8)
  valu_insts_per_simd_cycle = SQ_INSTS_VALU / (1024 x GRBM_GUI_ACTIVE / 8)   (wave instructions issued per SIMD
                              per cycle: at a 2-4 cycle issue cost per wave64 instruction, ~0.4 is a full VALU port)
Algorithmic HBM bytes per pixel: XORWOW 24 B state in + 24 B out + 4 B RGBA8; Philox 4 B; config 5 (progressive)
adds the float4 accumulator read and written (32 B)."""
import collections, csv, glob, json, os, sys

CONFIG = "c2"
if len(sys.argv) > 2 and sys.argv[1] == "--config":
    CONFIG = sys.argv[2]
    del sys.argv[1:3]
PIXELS = {"c2": 1920 * 1080, "c3": 3840 * 2160, "c4": 7680 * 4320, "c5": 1920 * 1080}[CONFIG]
ACCUM = 16 if CONFIG == "c5" else 0  # c5: each frame restarts the accumulation (camera moves): float4 written, not read


def passes(out):
    res = {}
    for d in sorted(glob.glob(os.path.join(out, "g*"))):
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        rows = [r for r in csv.DictReader(open(files[0])) if "render_kernel" in r["Kernel_Name"]]
        last = max(int(r["Dispatch_Id"]) for r in rows)
        acc = collections.defaultdict(float)
        for r in rows:
            if int(r["Dispatch_Id"]) == last:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
                kernel = r["Kernel_Name"]
        res.update(acc)
        res["kernel"] = kernel
    return res


def summary(out, rng):
    p = passes(out)
    gui = p["GRBM_GUI_ACTIVE"] / 8.0  # the traffic passes each carry it; the last one read wins (same launch shape)
    read = p["FETCH_SIZE"] * 1024.0 * 2.0
    write = p["WRITE_SIZE"] * 1024.0
    return {
        "kernel": p["kernel"],
        "rng": rng,
        "FETCH_SIZE_KB": p["FETCH_SIZE"],
        "WRITE_SIZE_KB": p["WRITE_SIZE"],
        "hbm_read_bytes_corrected": read,
        "hbm_write_bytes": write,
        "hbm_bytes_per_launch": read + write,
        "algorithmic_bytes_per_launch": PIXELS * ((52 if rng == "xorwow" else 4) + ACCUM),
        "valu_lane_utilization": round(p["SQ_THREAD_CYCLES_VALU"] / (64.0 * p["SQ_ACTIVE_INST_VALU"]), 4),
        "avg_waves_per_simd": round(4.0 * p["SQ_WAVE_CYCLES"] / (1024.0 * gui), 3),
        "ta_busy_frac_per_cu": round(p["TA_TA_BUSY_sum"] / 256.0 / gui, 4),
        "sq_insts_valu": int(p["SQ_INSTS_VALU"]),
        "valu_insts_per_simd_cycle": round(p["SQ_INSTS_VALU"] / (1024.0 * gui), 4),
        "gpu_cycles": int(gui),
    }


xorwow, philox = summary(sys.argv[1], "xorwow"), summary(sys.argv[2], "philox")
soa = summary(sys.argv[3], "xorwow") if len(sys.argv) > 3 else None
out = {
    "command": "rocprofv3 --pmc <one group per pass: FETCH_SIZE | WRITE_SIZE | SQ_* | TA_*> --kernel-include-regex "
               f"render_kernel -- python3 tools/one_frame.py --config {CONFIG} --variant -1 --frames 3 [--rng philox | "
               f"--state-layout soa]  (tools/profile_pmc.sh, tools/pmc_groups_traffic.txt; config {CONFIG}; last, warm "
               "dispatch; tools/pmc_bench_json.py)",
    "config": CONFIG,
    "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 reports 1/2 of wide reads). Algorithmic bytes: "
            "XORWOW mode 24 B state in + 24 B out + 4 B RGBA8 per pixel; the kernel touches 24 of each 48-B "
            "curandState (the reference layout), so whole lines move. Philox mode: 4 B per pixel; the 8x8 tile "
            "per wave writes 32-B row segments, so partial-line writes inflate WRITE_SIZE. soa: the same XORWOW "
            "streams in six uint32 planes (RT_FLAG_STATE_SOA), 24 B read + 24 B written per pixel with coalesced "
            "4-B accesses.",
    **xorwow,
    "philox": philox,
}
if soa:
    out["soa"] = dict(soa, state_layout="soa")
print(json.dumps(out, indent=1))
