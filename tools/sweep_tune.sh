#!/bin/bash
# Sweep one rt_set_tuning key through bench.py (same box, alternating values, REPS rounds).
#   bash tools/sweep_tune.sh "<bench args>" <key> <v1> <v2> ...      e.g. bash tools/sweep_tune.sh "--config c5 --steps 50" 0 24 32 40
#   EXTRA_TUNE=k=v[,k=v]: further rt_set_tuning overrides held fixed during the sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
ARGS=$1; KEY=$2; shift 2
for r in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $ARGS --tune ${EXTRA_TUNE:+$EXTRA_TUNE,}$KEY=$v \
      > gpurun_out/sweep.log 2>&1 || { tail -5 gpurun_out/sweep.log; exit 3; }
    python - "$KEY" "$v" "$r" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/sweep.log").read().strip().splitlines()[-1])
print(f"key {sys.argv[1]} = {sys.argv[2]} rep {sys.argv[3]}: kernel_ms {d['kernel_ms']} ms_per_step {d['ms_per_step']}", flush=True)
PY
  done
done
