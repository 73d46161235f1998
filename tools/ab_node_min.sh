#!/bin/bash
# A/B of RT_TUNE_NODE_MIN (key 11) against the tree before the knob (ab_src/render_base.hip = git show <parent>:...),
# then the cap x threshold grid with the leaf-break default.  Same box, bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/ab_variants_build.sh base=ab_src/render_base.hip > gpurun_out/abbuild.log 2>&1 || exit 3
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'])"
}
for r in 1 2; do
  one /tmp/ablib/base.so "c2 base" "--steps 20 --warmup 3"
  for X in 0 16 24 32 40; do one cudaraytracer_amd/librt_hip.so "c2 node_min=$X" "--steps 20 --warmup 3 --tune 11=$X"; done
done
for cap in 48 56 64; do for thr in 40 48 56; do one cudaraytracer_amd/librt_hip.so "c2 cap=$cap thr=$thr" "--steps 20 --warmup 3 --tune 9=$cap,0=$thr"; done; done
