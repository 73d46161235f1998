#!/bin/bash
# C5 same-box A/B of the persistent queue knobs through bench.py lines (13 = RT_TUNE_QUEUE_PREFETCH, 7 = RT_TUNE_QUEUE_CHUNK).
set -u
for rep in 1 2 3; do
  for t in "" "13=32,7=128" "13=32"; do
    timeout -k 10 200 python bench.py --config c5 --steps 20 --warmup 4 --no-cpu-baseline ${t:+--tune $t} > gpurun_out/ab_c5.log 2>&1 || exit 4
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_c5.log').read().strip().splitlines()[-1]); print('tune=[$t]', d['ms_per_step'], d['kernel_ms'])"
  done
done
