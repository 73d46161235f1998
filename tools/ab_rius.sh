#!/bin/bash
# A/B of the resumable RandomInUnitSphere in the v3 kernels (key 11 = attempts per shading pass, 0 = unbounded) on C2
# and C3, and of the threshold rule for deferred lanes (lower the regeneration threshold by the number of deferred
# lanes, or "nothr": count them as waiting lanes).  v3 kept no deferral (C2 loses at every cap, profiles/
# r04a_ab_rius_v3.txt), so both builds come from the commit that had it (099739c).  Same box, bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
[ -d ab_src/tree_rius_v3 ] || bash tools/ab_prepare.sh rius_v3 099739c || exit 3
rm -rf ab_src/tree_rius_v3_nothr && cp -r ab_src/tree_rius_v3 ab_src/tree_rius_v3_nothr && rm -rf ab_src/tree_rius_v3_nothr/build
sed -i 's/thr = thr > deferred + 1u ? thr - deferred : 1u;/(void)deferred;/' ab_src/tree_rius_v3_nothr/cudaraytracer_amd/csrc/render.hip
bash tools/ab_variants_build.sh rius=@rius_v3 nothr=@rius_v3_nothr > gpurun_out/abbuild.log 2>&1 || { tail -5 gpurun_out/abbuild.log; exit 3; }
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'], d['rays_per_frame'], flush=True)"
}
LIB=/tmp/ablib/rius.so
for r in 1 2; do
  for K in ${KS:-0 1 2 3 4 6}; do one $LIB "c2 trips=$K" "--steps 20 --warmup 3 --tune 11=$K"; done
  for K in 1 2 3; do one /tmp/ablib/nothr.so "c2 nothr trips=$K" "--steps 20 --warmup 3 --tune 11=$K"; done
done
for r in 1 2; do
  for K in ${KS:-0 1 2 3 4 6}; do one $LIB "c3 trips=$K" "--config c3 --steps 2 --warmup 1 --tune 11=$K"; done
  for K in 1 2 3; do one /tmp/ablib/nothr.so "c3 nothr trips=$K" "--config c3 --steps 2 --warmup 1 --tune 11=$K"; done
done
for K in 0 4 8; do
  one $LIB "c2 philox trips=$K" "--steps 20 --warmup 3 --rng philox --tune 11=$K"
  one $LIB "c3 philox trips=$K" "--config c3 --steps 2 --warmup 1 --rng philox --tune 11=$K"
done
