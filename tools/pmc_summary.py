"""Sum rocprofv3 counter_collection.csv values per counter for one dispatch of the render kernel (the last
one by default: with --frames N the adaptive tile order is in effect from the second frame).
    python tools/pmc_summary.py <profile_pmc.sh out dir> [--dispatch first|last]"""
import collections, csv, glob, json, os, sys

out = sys.argv[1]
which = sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--dispatch" else "last"
res = {}
for d in sorted(glob.glob(os.path.join(out, "g*"))):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        continue
    rows = [r for r in csv.DictReader(open(files[0])) if "render_kernel" in r["Kernel_Name"]]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    pick = ids[-1] if which == "last" else ids[0]
    acc = collections.defaultdict(float)
    dur = None
    for r in rows:
        if int(r["Dispatch_Id"]) == pick:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    res[os.path.basename(d)] = {"dispatch": pick, "ms": dur, **{k: v for k, v in acc.items()}}
print(json.dumps(res, indent=1))
