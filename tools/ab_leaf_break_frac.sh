#!/bin/bash
# (records the A/B of a knob that is not in the product source)
# A/B of RT_TUNE_LEAF_BREAK_FRAC (key 11) against the tree before the knob (ab_src/render_base.hip = git show
# <parent>:cudaraytracer_amd/csrc/render.hip), same box, bench.py C2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/ab_variants_build.sh base=ab_src/render_base.hip > gpurun_out/abbuild.log 2>&1 || exit 3
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'])"
}
for r in 1 2; do
  one /tmp/ablib/base.so "c2 base" "--steps 20 --warmup 3"
  for F in 0 4 8 12 16; do one cudaraytracer_amd/librt_hip.so "c2 frac=$F" "--steps 20 --warmup 3 --tune 11=$F"; done
done
