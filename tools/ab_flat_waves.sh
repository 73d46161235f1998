#!/bin/bash
# Flat kernel (variant 5) occupancy: __launch_bounds__ waves per SIMD of the untextured build (kFlatWaves) x the
# reference replay inlined or called (ref_trace).  Same box, bench.py C3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SRC=cudaraytracer_amd/csrc/render.hip
INL='s/__device__ __noinline__ HitOut ref_trace/__device__ __forceinline__ HitOut ref_trace/'
specs=()
for W in 8 7 6 5; do
  [ $W = 8 ] || specs+=("call_w$W=$SRC:s/constexpr int kFlatWaves = 8;/constexpr int kFlatWaves = $W;/")
  specs+=("inline_w$W=$SRC:s/constexpr int kFlatWaves = 8;/constexpr int kFlatWaves = $W;/;$INL")
done
bash tools/ab_variants_build.sh "${specs[@]}" > gpurun_out/abbuild.log 2>&1 || { tail -5 gpurun_out/abbuild.log; exit 3; }
cp cudaraytracer_amd/librt_hip.so /tmp/ablib/call_w8.so
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'], d['rays_per_frame'], flush=True)"
}
for r in 1 2; do
  for W in 8 7 6 5; do
    for k in call inline; do one /tmp/ablib/${k}_w$W.so "c3 flat $k W=$W" "--config c3 --steps 2 --warmup 1 --variant 5 --tune 11=4"; done
  done
done
