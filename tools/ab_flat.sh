#!/bin/bash
# Flat kernel (variant 5) against v3 compact (variant 3) on the small-scene configs, and its RandomInUnitSphere cap
# (RT_TUNE_RIUS_TRIPS, key 11).  Same box, bench.py lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
one() {  # label args
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $2 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$1', d['kernel_ms'], d['ms_per_step'], d['rays_per_frame'], flush=True)"
}
for r in 1 2; do
  one "c3 v3" "--config c3 --steps 2 --warmup 1 --variant 3"
  for K in ${KS:-0 1 2 3 4}; do one "c3 flat trips=$K" "--config c3 --steps 2 --warmup 1 --variant 5 --tune 11=$K"; done
done
one "c3 philox v3" "--config c3 --steps 2 --warmup 1 --variant 3 --rng philox"
for K in 0 4; do one "c3 philox flat trips=$K" "--config c3 --steps 2 --warmup 1 --variant 5 --rng philox --tune 11=$K"; done
for v in 4 6 -1; do one "c5 variant $v" "--config c5 --steps 20 --warmup 4 --variant $v"; done
one "c2 auto (488 spheres: v3)" "--steps 10 --warmup 2"
