#!/bin/bash
# Where the flat kernel's extra HBM bytes on C3 come from: FETCH_SIZE and WRITE_SIZE (one rocprofv3 pass each) of the
# product against a build without the exactness replay ("noexact": the check's result ignored, so no ref_trace call
# and no private stack or call frame), Philox mode (no RNG state: only RGBA8 is algorithmic).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_replay; export TMPDIR=/tmp
SRC=cudaraytracer_amd/csrc/render.hip
bash tools/ab_variants_build.sh "noexact=$SRC:s/if (tie || nan || edge || t_best != t_best) {/if (false) {/" \
  > gpurun_out/abbuild.log 2>&1 || { tail -5 gpurun_out/abbuild.log; exit 3; }
cp cudaraytracer_amd/librt_hip.so /tmp/ablib/product.so
for v in product noexact; do
  for c in FETCH_SIZE WRITE_SIZE; do
    RT_HIP_LIB=/tmp/ablib/$v.so timeout -k 10 120 rocprofv3 --pmc $c --kernel-include-regex render_kernel \
      -d gpurun_out/pmc_replay/${v}_$c -o p --output-format csv -- python3 tools/one_frame.py --config c3 --frames 2 --rng philox \
      > gpurun_out/pmc_replay/${v}_$c.log 2>&1 || exit $?
    python - "$v" "$c" <<'PY'
import csv, glob, sys
v, c = sys.argv[1], sys.argv[2]
rows = [r for f in glob.glob(f"gpurun_out/pmc_replay/{v}_{c}/**/p_counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
last = max(int(r["Dispatch_Id"]) for r in rows)
val = sum(float(r["Counter_Value"]) for r in rows if int(r["Dispatch_Id"]) == last)
print(f"c3 philox {v} {c} {val:.0f} KB (dispatch {last})", flush=True)
PY
  done
done
