#!/bin/bash
# PMC latency/occupancy groups for several variants: PMC_VARIANTS="13 16"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${PMC_VARIANTS:-13}; do
  PMC_GROUPS_FILE=tools/pmc_groups_latency.txt bash tools/profile_pmc.sh $v gpurun_out/lat$v || exit $?
  python3 tools/pmc_summary.py gpurun_out/lat$v > gpurun_out/lat$v.json || exit $?
done
echo done
