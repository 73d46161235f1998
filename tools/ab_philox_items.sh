#!/bin/bash
# Philox sample items in v3 and the flat kernel (a full tile's 64 x spp samples handed to whichever lane's path ended)
# against the same build with items off (every lane renders its own pixel's samples in order; the same Philox windows and fixed-point sums,
# so the same image).  Same box, bench.py C2 Philox lines, 3 rounds, then C4 Philox and XORWOW C2 as controls.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SRC=cudaraytracer_amd/csrc/render.hip
bash tools/ab_variants_build.sh "noitems=$SRC:s/const bool items = kItemsBuild \&\& P.spp > 0/const bool items = false \&\& P.spp > 0/" \
  > gpurun_out/abbuild.log 2>&1 || { tail -5 gpurun_out/abbuild.log; exit 3; }
cp cudaraytracer_amd/librt_hip.so /tmp/ablib/product.so
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'], d['rays_per_frame'], flush=True)"
}
for r in 1 2 3; do
  for v in noitems product; do
    one /tmp/ablib/$v.so "c2 philox $v" "--steps 10 --warmup 2 --rng philox"
  done
done
for v in noitems product; do one /tmp/ablib/$v.so "c2 xorwow $v" "--steps 10 --warmup 2"; done
for v in noitems product; do one /tmp/ablib/$v.so "c4 philox $v" "--config c4 --steps 2 --warmup 1 --rng philox"; done
for r in 1 2; do
  for v in noitems product; do one /tmp/ablib/$v.so "c3 philox $v" "--config c3 --steps 2 --warmup 1 --rng philox"; done
done
for v in noitems product; do one /tmp/ablib/$v.so "c3 xorwow $v" "--config c3 --steps 2 --warmup 1"; done
