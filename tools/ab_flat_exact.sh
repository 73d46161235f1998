#!/bin/bash
# Cost of the flat kernels' exactness check (tie / NaN / box-face test + reference replay, render.hip flat_trace):
# the product build against a build without it ("noexact": the replay condition patched to false, which lets the
# compiler drop the checks).  Same box, bench.py C3 / C5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/ab_variants_build.sh \
  'noexact=cudaraytracer_amd/csrc/render.hip:s/if (tie || nan || edge || t_best != t_best) {/if (false) {/' \
  'inline=cudaraytracer_amd/csrc/render.hip:s/__device__ __noinline__ HitOut ref_trace/__device__ __forceinline__ HitOut ref_trace/' \
  > gpurun_out/abbuild.log 2>&1 || { tail -5 gpurun_out/abbuild.log; exit 3; }
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'], d['rays_per_frame'], flush=True)"
}
LIB=cudaraytracer_amd/librt_hip.so
for r in 1 2; do
  one $LIB "c3 exact flat K=4" "--config c3 --steps 2 --warmup 1 --variant 5 --tune 11=4"
  one /tmp/ablib/noexact.so "c3 noexact flat K=4" "--config c3 --steps 2 --warmup 1 --variant 5 --tune 11=4"
  one /tmp/ablib/inline.so "c3 inline flat K=4" "--config c3 --steps 2 --warmup 1 --variant 5 --tune 11=4"
  one $LIB "c5 exact persistent flat" "--config c5 --steps 20 --warmup 4 --variant 6"
  one /tmp/ablib/noexact.so "c5 noexact persistent flat" "--config c5 --steps 20 --warmup 4 --variant 6"
  one /tmp/ablib/inline.so "c5 inline persistent flat" "--config c5 --steps 20 --warmup 4 --variant 6"
  one $LIB "c5 v4" "--config c5 --steps 20 --warmup 4 --variant 4"
done
