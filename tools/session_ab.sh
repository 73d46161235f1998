#!/bin/bash
# Parity tests of selected variants + interleaved A/B timing (tools/ab_variants.py) on configs c2/c3/c5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x --timeout 300 ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for c in ${AB_CONFIGS:-c2}; do
  timeout -k 10 300 python tools/ab_variants.py --config $c --variants ${AB_VARIANTS:-13,22} --rounds ${AB_ROUNDS:-3} ${AB_EXTRA:-} > gpurun_out/ab_$c.log 2>&1 || exit $?
done
echo done
