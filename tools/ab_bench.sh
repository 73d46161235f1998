#!/bin/bash
# Same-box A/B of librt_hip.so builds through bench.py (one process per library and repetition, alternating).
#   bash tools/ab_bench.sh "<bench args>" <libA.so> <libB.so> ...     (REPS=2; prints kernel_ms and ms_per_step)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
ARGS=$1; shift
for r in $(seq 1 ${REPS:-2}); do
  for lib in "$@"; do
    RT_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $ARGS \
      > gpurun_out/ab_bench.log 2>&1 || { tail -5 gpurun_out/ab_bench.log; exit 3; }
    python - "$lib" "$r" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_bench.log").read().strip().splitlines()[-1])
print(f"{sys.argv[1]} rep {sys.argv[2]}: kernel_ms {d['kernel_ms']} ms_per_step {d['ms_per_step']} rays {d['rays_per_frame']}", flush=True)
PY
  done
done
