#!/bin/bash
# Persistent flat kernel (variant 6) occupancy on C5: the textured builds under __launch_bounds__(64, W) for W = 6
# and 8 (the compiler holds them to 80 / 64 VGPRs, spilling the rest) against the product's unbounded build (93
# VGPRs, 5 waves per SIMD); the persistent grid follows the occupancy query.  Same box, bench.py C5 lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SRC=cudaraytracer_amd/csrc/render.hip
P='dev::render_kernel_flat_persistent<false, true, PH, 1>;'
bash tools/ab_variants_build.sh "w6=$SRC:s/$P/dev::render_kernel_flat_persistent<false, true, PH, 6>;/" \
  "w8=$SRC:s/$P/dev::render_kernel_flat_persistent<false, true, PH, 8>;/" \
  > gpurun_out/abbuild.log 2>&1 || { tail -5 gpurun_out/abbuild.log; exit 3; }
cp cudaraytracer_amd/librt_hip.so /tmp/ablib/product.so
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'], d['rays_per_frame'], flush=True)"
}
for r in 1 2 3; do
  for v in product w6 w8; do
    one /tmp/ablib/$v.so "c5 $v" "--config c5 --steps 40 --warmup 4 --variant 6"
    one /tmp/ablib/$v.so "c5 philox $v" "--config c5 --steps 40 --warmup 4 --variant 6 --rng philox"
  done
done
for v in product w6 w8; do
  RT_HIP_LIB=/tmp/ablib/$v.so timeout -k 10 200 python tools/v4_timeline.py --variant 6 --frames 8 --cases 1 --detail 2>/dev/null | head -2 | sed "s/^/$v /"
done
