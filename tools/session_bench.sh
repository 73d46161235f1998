#!/bin/bash
# Headline bench + rocprofv3 kernel summary + PMC HBM traffic + per-config timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || exit $?
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex render_kernel -d gpurun_out/pmc_bench_$grp -o p --output-format csv -- python3 tools/one_frame.py --frames 1 > gpurun_out/pmc_bench_$grp.log 2>&1 || exit $?
done
timeout -k 10 300 python tools/bench_configs.py > gpurun_out/configs.log 2>&1 || exit $?
echo done
