#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, no traces), for one kernel variant.
# usage: bash tools/profile_pmc.sh <variant> <outdir>    (PMC_GROUPS_FILE=<file>: one group per line)
set -u
V=${1:-1}; OUT=${2:-gpurun_out/pmc}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p "$OUT"; export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
DEFAULT_GROUPS='SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS
FETCH_SIZE
WRITE_SIZE
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum
TA_BUSY_avr TA_TA_BUSY_sum'
if [ -n "${PMC_GROUPS_FILE:-}" ]; then GROUPS_TEXT=$(cat "$PMC_GROUPS_FILE"); else GROUPS_TEXT=$DEFAULT_GROUPS; fi
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --kernel-include-regex render_kernel -d "$OUT/g$i" -o p --output-format csv -- python3 tools/one_frame.py --variant "$V" --frames 1 ${ONE_FRAME_ARGS:-} > "$OUT/g$i.log" 2>&1
  rc=$?; echo "group $i ($group) rc=$rc" >> "$OUT/summary.txt"
  if [ $rc -ge 124 ]; then exit $rc; fi
done <<< "$GROUPS_TEXT"
echo pmc-done
