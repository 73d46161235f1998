#!/bin/bash
# Flat kernels' exactness check from the per-record box table (pack_flat_box) with the NaN rule moved to one per-ray
# test, against round 4's per-lane-selected check with per-primitive NaN masks (revision 521115e, exported by
# tools/ab_prepare.sh r4base 521115e).  Same box, bench.py C3 (flat) and C5 (persistent flat), 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
[ -d ab_src/tree_r4base ] || bash tools/ab_prepare.sh r4base 521115e || exit 3
[ -d ab_src/tree_boxes1 ] || bash tools/ab_prepare.sh boxes1 1b8c328 || exit 3
bash tools/ab_variants_build.sh "r4base=@r4base" "boxes1=@boxes1" > gpurun_out/abbuild.log 2>&1 || { tail -5 gpurun_out/abbuild.log; exit 3; }
cp cudaraytracer_amd/librt_hip.so /tmp/ablib/product.so
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'], d['rays_per_frame'], flush=True)"
}
for r in 1 2 3; do
  for v in ${VARIANTS:-r4base boxes1 product}; do
    one /tmp/ablib/$v.so "c3 flat $v" "--config c3 --steps 2 --warmup 1"
    one /tmp/ablib/$v.so "c5 pflat $v" "--config c5 --steps 20 --warmup 4"
  done
done
for v in ${VARIANTS:-r4base boxes1 product}; do one /tmp/ablib/$v.so "c3 flat philox $v" "--config c3 --steps 2 --warmup 1 --rng philox"; done
