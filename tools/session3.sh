#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python tools/ab_variants.py --variants ${AB_VARIANTS:-6,8,9,11,12} --thresholds ${AB_THR:-32,48} --leafmax ${AB_LM:-4} --pwaves ${AB_PW:-0} --rounds 3 > gpurun_out/ab.log 2>&1 || exit $?
timeout -k 10 300 python tools/simd_eff.py c2 ${SIMD_VARIANTS:-8,11,12} > gpurun_out/simd.log 2>&1 || exit $?
if [ -n "${PMC_VARIANT:-}" ]; then bash tools/profile_pmc.sh $PMC_VARIANT gpurun_out/pmc$PMC_VARIANT || exit $?; fi
echo done
