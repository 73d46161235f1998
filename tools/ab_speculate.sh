#!/bin/bash
# v3 speculative traversal (ab_src/v3_speculate.patch: a lane that holds its postponed leaf and meets a second one
# keeps traversing; the second leaf takes the stack slot of the node it continues with) against the product.
# Same box, bench.py C2 (XORWOW and Philox) and the COUNT_TESTS phase counters (tools/simd_eff.py), 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
[ -d ab_src/tree_spec ] || bash tools/ab_prepare.sh spec HEAD ab_src/v3_speculate.patch || exit 3
bash tools/ab_variants_build.sh "spec=@spec" > gpurun_out/abbuild.log 2>&1 || { tail -5 gpurun_out/abbuild.log; exit 3; }
cp cudaraytracer_amd/librt_hip.so /tmp/ablib/product.so
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'], d['rays_per_frame'], flush=True)"
}
for r in 1 2 3; do
  for v in product spec; do
    one /tmp/ablib/$v.so "c2 $v" "--steps 10 --warmup 2"
  done
done
for v in product spec; do one /tmp/ablib/$v.so "c2 philox $v" "--steps 10 --warmup 2 --rng philox"; done
for v in product spec; do
  RT_HIP_LIB=/tmp/ablib/$v.so timeout -k 10 200 python tools/simd_eff.py c2 3 2>/dev/null | sed "s/^/$v /"
done
