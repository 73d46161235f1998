#!/bin/bash
# C5 same-box A/B of the persistent queue / grid knobs through bench.py lines, alternating (REPS rounds):
# 13 = RT_TUNE_QUEUE_PREFETCH, 7 = RT_TUNE_QUEUE_CHUNK, 2 = RT_TUNE_PERSISTENT_WAVES.  Prints ms_per_step kernel_ms.
#   TUNES="|13=32,7=128|13=32" bash tools/ab_c5_queue.sh
set -u
IFS='|' read -r -a SETS <<< "${TUNES:-|13=32,7=128|13=32}"
for rep in $(seq 1 ${REPS:-3}); do
  for t in "${SETS[@]}"; do
    timeout -k 10 200 python bench.py --config c5 --steps 20 --warmup 4 --no-cpu-baseline ${t:+--tune $t} > gpurun_out/ab_c5.log 2>&1 || exit 4
    python -c "import json; d=json.loads(open('gpurun_out/ab_c5.log').read().strip().splitlines()[-1]); print('tune=[$t]', d['ms_per_step'], d['kernel_ms'])"
  done
done
