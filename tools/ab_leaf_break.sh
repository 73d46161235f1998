#!/bin/bash
# A/B of the RT_TUNE_LEAF_BREAK knob (key 10) against the tree before it (commit 36f2cee, the parent of 9ed3177 that
# added it).  Same box, bench.py C2 and C3 (profiles/r03r_ab_leaf_break.txt).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
[ -d ab_src/tree_leafbreak_base ] || bash tools/ab_prepare.sh leafbreak_base 36f2cee || exit 3
bash tools/ab_variants_build.sh base=@leafbreak_base > gpurun_out/abbuild.log 2>&1 || { tail -5 gpurun_out/abbuild.log; exit 3; }
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'])"
}
for r in 1 2; do
  one /tmp/ablib/base.so "c2 base" "--steps 20 --warmup 3"
  for K in 0 1 2 4 8; do one cudaraytracer_amd/librt_hip.so "c2 leafbreak=$K" "--steps 20 --warmup 3 --tune 10=$K"; done
done
for K in 0 2; do one cudaraytracer_amd/librt_hip.so "c3 leafbreak=$K" "--config c3 --variant 3 --steps 2 --warmup 1 --tune 10=$K"; done
