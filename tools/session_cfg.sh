#!/bin/bash
# Config-3/5 timings and a c2 A/B for several variants: CFG_VARIANTS="13,21" AB_VARIANTS="13,21" AB_ROUNDS=6
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python tools/bench_configs.py --variants ${CFG_VARIANTS:-13} > gpurun_out/cfg.log 2>&1 || exit $?
timeout -k 10 400 python tools/ab_variants.py --variants ${AB_VARIANTS:-13} --thresholds 40 --leafmax 4 --rounds ${AB_ROUNDS:-6} > gpurun_out/ab.log 2>&1 || exit $?
echo done
