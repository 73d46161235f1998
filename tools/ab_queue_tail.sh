#!/bin/bash
# Persistent kernels' queue near a head's end: "exactneed" takes exactly as many work indices as the wave's lanes wait
# for, the product 64 (round 3's rule, kept: exact-need lost 8-10 %, profiles/r04e_ab_c5_prefetch.txt).  Same box,
# bench.py C5 (persistent flat) and v4 on C5, then the timelines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SRC=cudaraytracer_amd/csrc/render.hip
bash tools/ab_variants_build.sh "exactneed=$SRC:s/const uint32_t want = head_left > 4u \* P.work_chunk ? P.work_chunk : 64u;/const uint32_t want = head_left > 4u * P.work_chunk ? P.work_chunk : (uint32_t)__popcll(needm);/" \
  > gpurun_out/abbuild.log 2>&1 || { tail -5 gpurun_out/abbuild.log; exit 3; }
cp cudaraytracer_amd/librt_hip.so /tmp/ablib/product.so
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'], d['rays_per_frame'], flush=True)"
}
for r in 1 2 3; do
  for v in product exactneed; do
    one /tmp/ablib/$v.so "c5 pflat $v" "--config c5 --steps 40 --warmup 4 --variant 6"
    one /tmp/ablib/$v.so "c5 v4 $v" "--config c5 --steps 40 --warmup 4 --variant 4"
  done
done
for v in product exactneed; do
  RT_HIP_LIB=/tmp/ablib/$v.so timeout -k 10 200 python tools/v4_timeline.py --variant 6 --frames 8 2>/dev/null | head -1 | sed "s/^/$v /"
done
