set -u
# (A/B of the RT_TUNE_LEAF_BREAK knob against the tree before it: ab_src/render_base.hip = git show <parent>:cudaraytracer_amd/csrc/render.hip)
bash tools/ab_variants_build.sh base=ab_src/render_base.hip > gpurun_out/abbuild.log 2>&1 || exit 3
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'])"
}
for r in 1 2; do
  one /tmp/ablib/base.so "c2 base" "--steps 20 --warmup 3"
  for K in 0 1 2 4 8; do one cudaraytracer_amd/librt_hip.so "c2 leafbreak=$K" "--steps 20 --warmup 3 --tune 10=$K"; done
done
for K in 0 2; do one cudaraytracer_amd/librt_hip.so "c3 leafbreak=$K" "--config c3 --steps 2 --warmup 1 --tune 10=$K"; done
