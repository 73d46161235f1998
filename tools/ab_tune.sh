#!/bin/bash
# Same-box A/B of rt_set_tuning settings through bench.py (one process per setting and repetition, alternating).
#   bash tools/ab_tune.sh "<bench args>" "<tune A>" "<tune B>" ...   (REPS=3; a tune is key=value[,key=value] or "-")
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
ARGS=$1; shift
for r in $(seq 1 ${REPS:-3}); do
  for tune in "$@"; do
    t=$tune; [ "$t" = "-" ] && t=""
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $ARGS --tune "$t" \
      > gpurun_out/ab_tune.log 2>&1 || { tail -5 gpurun_out/ab_tune.log; exit 3; }
    python - "$tune" "$r" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_tune.log").read().strip().splitlines()[-1])
print(f"tune {sys.argv[1]} rep {sys.argv[2]}: kernel_ms {d['kernel_ms']} ms_per_step {d['ms_per_step']} rays {d['rays_per_frame']}", flush=True)
PY
  done
done
