#!/bin/bash
# Traffic/SIMD-efficiency PMC passes (tools/pmc_groups_traffic.txt, one counter group per rocprofv3 run) of the
# default kernel for each config in $CONFIGS and each RNG mode / state layout, then the per-config summaries
# profiles read by bench.py.  usage (repo root, on the GPU box): CONFIGS="c2 c3 c5" bash tools/pmc_configs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cfg in ${CONFIGS:-c2 c3 c5}; do
  F=3; [ $cfg = c5 ] && F=6  # c5: past the automatic v3/v4 trial frames
  for mode in xorwow philox soa; do
    case $mode in
      xorwow) a="--config $cfg --frames $F" ;;
      philox) a="--config $cfg --frames $F --rng philox" ;;
      soa)    a="--config $cfg --frames $F --state-layout soa" ;;
    esac
    ONE_FRAME_ARGS="$a" PMC_GROUPS_FILE=tools/pmc_groups_traffic.txt bash tools/profile_pmc.sh -1 gpurun_out/pmc_$cfg/$mode \
      > /dev/null || exit $?
    echo "$cfg $mode: $(tail -4 gpurun_out/pmc_$cfg/$mode/summary.txt | tr '\n' ' ')"
  done
  python tools/pmc_bench_json.py --config $cfg gpurun_out/pmc_$cfg/xorwow gpurun_out/pmc_$cfg/philox \
    gpurun_out/pmc_$cfg/soa > gpurun_out/pmc_${cfg}_n1.json || exit $?
done
echo pmc-configs-done
