#!/bin/bash
# C5 (1 spp progressive, persistent flat kernel, variant 6): prefetch of the next pixel's XORWOW state (kFlatPrefetch
# bit 0, the product) stopped once the wave's queue head is below 1/kPrefetchStop of its range (8, the product; 2, 4,
# never), against no prefetch.  (Round 4's first A/B also had the accumulator prefetch, bit 1: slower.)  Same box, bench.py C5 lines
# (XORWOW and Philox), then the wave timeline of each build (tools/v4_timeline.py --variant 6).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SRC=cudaraytracer_amd/csrc/render.hip
bash tools/ab_variants_build.sh "pf0=$SRC:s/constexpr int kFlatPrefetch = 1;/constexpr int kFlatPrefetch = 0;/" \
  "pf1stop2=$SRC:s/constexpr uint32_t kPrefetchStop = 8;/constexpr uint32_t kPrefetchStop = 2;/" \
  "pf1stop4=$SRC:s/constexpr uint32_t kPrefetchStop = 8;/constexpr uint32_t kPrefetchStop = 4;/" \
  "pf1always=$SRC:s/constexpr uint32_t kPrefetchStop = 8;/constexpr uint32_t kPrefetchStop = 0xffffffffu;/" \
  > gpurun_out/abbuild.log 2>&1 || { tail -5 gpurun_out/abbuild.log; exit 3; }
cp cudaraytracer_amd/librt_hip.so /tmp/ablib/pf1stop8.so
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'], d['rays_per_frame'], flush=True)"
}
for r in 1 2 3; do
  for v in pf0 pf1stop2 pf1stop4 pf1stop8 pf1always; do one /tmp/ablib/$v.so "c5 $v" "--config c5 --steps 40 --warmup 4 --variant 6"; done
done
for v in pf0 pf1stop8; do one /tmp/ablib/$v.so "c5 philox $v" "--config c5 --steps 40 --warmup 4 --variant 6 --rng philox"; done
for v in pf0 pf1stop8 pf1always; do
  RT_HIP_LIB=/tmp/ablib/$v.so timeout -k 10 200 python tools/v4_timeline.py --variant 6 --frames 8 2>/dev/null | head -2 | sed "s/^/$v /"
done
