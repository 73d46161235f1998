#!/bin/bash
# A/B of builds of librt_hip.so on the same GPU box: runs tools/ab_variants.py against each library in
# turn (ROUNDS alternations).  Usage (on the box): bash tools/ab_builds.sh <libA.so> <libB.so> [more.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    for c in ${AB_CONFIGS:-c2}; do
      echo "== $lib round $r" >> gpurun_out/ab_builds_$c.log
      RT_HIP_LIB=$lib timeout -k 10 300 python tools/ab_variants.py --config $c --variants ${AB_VARIANTS:-3} --rounds ${AB_ROUNDS:-3} ${AB_EXTRA:-} 2>&1 | grep -v amdgpu.ids >> gpurun_out/ab_builds_$c.log || exit $?
    done
  done
done
echo done
