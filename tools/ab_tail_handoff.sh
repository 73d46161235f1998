set -u
# (records the A/B of ab_src/tail_handoff.patch: apply it to render.hip before running; the product source has no hand-off)
bash tools/ab_variants_build.sh base=ab_src/render_base.hip > gpurun_out/abbuild.log 2>&1 || exit 3
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "tail_handoff" -x -q --timeout 120 --timeout-method thread > gpurun_out/tail_tests.log 2>&1
rc=$?; tail -2 gpurun_out/tail_tests.log; [ $rc -eq 0 ] || exit $rc
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'], d['rays_per_frame'])"
}
for r in 1 2; do
  one /tmp/ablib/base.so base ""
  for K in 0 8 16 24 32; do one cudaraytracer_amd/librt_hip.so "new K=$K" "--tune 9=$K"; done
done
