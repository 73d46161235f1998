#!/bin/bash
# Flat kernel XORWOW pixel pool (ab_src/flat_pixel_pool.patch: 4 tiles per wave, lanes take the pool's pixels as
# theirs finish; not kept) against the product, and the patched build with the pool off at run time (kFlatPoolTiles =
# 1: the same code, its register cost without the pool).  Same box, bench.py C3, 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SRC=cudaraytracer_amd/csrc/render.hip
[ -d ab_src/tree_pool ] || bash tools/ab_prepare.sh pool HEAD ab_src/flat_pixel_pool.patch || exit 3
[ -d ab_src/tree_pooloff ] || { bash tools/ab_prepare.sh pooloff HEAD ab_src/flat_pixel_pool.patch && \
  sed -i 's/constexpr uint32_t kFlatPoolTiles = 4;/constexpr uint32_t kFlatPoolTiles = 1;/' ab_src/tree_pooloff/cudaraytracer_amd/csrc/render.hip; } || exit 3
bash tools/ab_variants_build.sh "pool=@pool" "pooloff=@pooloff" > gpurun_out/abbuild.log 2>&1 || { tail -5 gpurun_out/abbuild.log; exit 3; }
cp cudaraytracer_amd/librt_hip.so /tmp/ablib/prepool.so
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'], d['rays_per_frame'], flush=True)"
}
for r in 1 2 3; do
  for v in prepool pooloff pool; do one /tmp/ablib/$v.so "c3 $v" "--config c3 --steps 2 --warmup 1"; done
done
for v in prepool pool; do one /tmp/ablib/$v.so "c3 philox $v" "--config c3 --steps 2 --warmup 1 --rng philox"; done
