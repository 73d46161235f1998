#!/bin/bash
# Cost of each part of the flat kernels' exactness check (render.hip flat_trace): product, without the box-face test
# ("noedge"), without the tie / NaN tracking ("notie"), without any ("noexact").  Same box, bench.py C3 and C5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SRC=cudaraytracer_amd/csrc/render.hip
bash tools/ab_variants_build.sh \
  "noedge=$SRC:s/^    if (hit >= 0) {$/    if (false) {/" \
  "notie=$SRC:s/if (tie || nan || edge || t_best != t_best) {/if (edge || t_best != t_best) {/" \
  "noexact=$SRC:s/if (tie || nan || edge || t_best != t_best) {/if (false) {/" \
  > gpurun_out/abbuild.log 2>&1 || { tail -5 gpurun_out/abbuild.log; exit 3; }
cp cudaraytracer_amd/librt_hip.so /tmp/ablib/product.so
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'], d['rays_per_frame'], flush=True)"
}
for r in 1 2; do
  for v in ${VARIANTS:-product noedge notie noexact}; do
    one /tmp/ablib/$v.so "c3 flat $v" "--config c3 --steps 2 --warmup 1 --variant 5 --tune 11=4"
    one /tmp/ablib/$v.so "c5 pflat $v" "--config c5 --steps 20 --warmup 4 --variant 6"
  done
done
