#!/bin/bash
# A/B of RT_TUNE_RIUS_TRIPS (key 11: RandomInUnitSphere attempts per v3 shading pass, 0 = unbounded) on C2 and C3,
# and of the threshold rule for deferred lanes (the product lowers the regeneration threshold by the number of
# deferred lanes; "nothr" counts them as waiting lanes instead: a sed patch built on the box).  Same box, bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/ab_variants_build.sh \
  'nothr=cudaraytracer_amd/csrc/render.hip:s/thr = thr > deferred + 1u ? thr - deferred : 1u;/(void)deferred;/' \
  > gpurun_out/abbuild.log 2>&1 || { tail -5 gpurun_out/abbuild.log; exit 3; }
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'], d['rays_per_frame'], flush=True)"
}
LIB=cudaraytracer_amd/librt_hip.so
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
