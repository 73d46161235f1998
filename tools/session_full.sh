#!/bin/bash
# End-of-milestone GPU session: parity tests, smoke, bench (+ rocprofv3 kernel stats), per-config timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || exit $?
timeout -k 10 400 python tools/bench_configs.py > gpurun_out/configs.log 2>&1 || exit $?
echo done
