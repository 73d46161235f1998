#!/bin/bash
# A/B of the tail hand-off experiment (ab_src/tail_handoff.patch: slow pixels of v3 handed to a second kernel, knob
# key 9 = pixels left per wave below which it hands off) against the tree it was written for (the parent of 1de7ba4).
# Same box, bench.py C2 (profiles/r03i_ab_tail_handoff.txt).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
[ -d ab_src/tree_handoff_base ] || bash tools/ab_prepare.sh handoff_base 1de7ba4^ || exit 3
[ -d ab_src/tree_handoff ] || bash tools/ab_prepare.sh handoff 1de7ba4^ ab_src/tail_handoff.patch || exit 3
bash tools/ab_variants_build.sh base=@handoff_base new=@handoff > gpurun_out/abbuild.log 2>&1 || { tail -5 gpurun_out/abbuild.log; exit 3; }
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'], d['rays_per_frame'])"
}
for r in 1 2; do
  one /tmp/ablib/base.so base ""
  for K in 0 8 16 24 32; do one /tmp/ablib/new.so "new K=$K" "--tune 9=$K"; done
done
