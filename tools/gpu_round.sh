#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel-trace summary.  Stops at the first GPU fault,
# abort, segfault or timeout (pytest rc 1 = test failures only, which does not stop the session).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_prof.log 2>&1 || exit $?
echo done
