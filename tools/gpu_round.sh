#!/bin/bash
# One GPU session (run through gpurun from the repo root): parity tests, smoke, bench + rocprofv3 kernel
# summary, per-config timings.  Every GPU step has its own time limit and the session stops at the first
# GPU fault, abort, segfault or timeout (pytest rc 1 = test failures only, which does not stop it).
#   STEPS="tests smoke bench prof benchcfg configs rehearse"   (default: tests smoke bench prof benchcfg)
#   PYTEST_ARGS=...   BENCH_ARGS=...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-tests smoke bench prof benchcfg}
for step in $STEPS; do
  case $step in
    tests)
      timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
        ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ;;
    smoke)
      timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || exit $? ;;
    bench)
      timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || exit $?
      tail -1 gpurun_out/bench.log ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- \
        python3 bench.py --no-cpu-baseline --no-config-lines ${BENCH_ARGS:-} > gpurun_out/bench_prof.log 2>&1 || exit $? ;;
    benchcfg)  # driver-shaped lines for BASELINE configs 3 and 5
      for cfg in c5 c3; do
        steps=${CFG_STEPS:-5}; [ $cfg = c5 ] && steps=${C5_STEPS:-20}  # C5's orbit: average 20 frames, as other_configs.c5
        timeout -k 10 400 python bench.py --config $cfg --steps $steps --warmup 2 ${BENCH_ARGS:-} \
          > gpurun_out/bench_$cfg.log 2>&1 || exit $?
        tail -1 gpurun_out/bench_$cfg.log
      done ;;
    selfcheck)  # bench.py --gpus 2 on a 1-GPU box must fail (no N=1 line)
      if timeout -k 10 120 python bench.py --gpus 2 --steps 1 --warmup 0 > gpurun_out/selfcheck.log 2>&1; then
        echo "selfcheck: --gpus 2 ran on one GPU" ; exit 3; fi
      tail -2 gpurun_out/selfcheck.log ;;
    rehearse)  # bench.py's self-launched N > 1 path with every rank on device 0 (gloo gather): C2 weak, C4 strong
      for n in ${REHEARSE_N:-2 4}; do
        for cfg in c2 c4; do
          timeout -k 10 400 python bench.py --gpus $n --steps 3 --warmup 1 --config $cfg --backend gloo \
            --share-gpu --no-cpu-baseline --no-philox-line > gpurun_out/rehearse_${cfg}_n$n.log 2>&1 || exit $?
          tail -1 gpurun_out/rehearse_${cfg}_n$n.log
        done
      done ;;
    configs)
      timeout -k 10 400 python tools/bench_configs.py ${CONFIGS_ARGS:-} > gpurun_out/configs.log 2>&1 || exit $?
      cat gpurun_out/configs.log | grep -v amdgpu.ids ;;
  esac
done
echo done
