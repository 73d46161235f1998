#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python tools/ab_variants.py --variants 1,6,8,9,10 --thresholds 16,32,40,48,56 --rounds 3 > gpurun_out/ab.log 2>&1 || exit $?
bash tools/profile_pmc.sh 8 gpurun_out/pmc8 || exit $?
echo done
