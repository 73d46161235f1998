#!/bin/bash
# Device assembly of render.hip (gfx950) and the body of one kernel.
#   bash tools/dump_isa.sh <mangled-kernel-symbol> [lines]   -> /tmp/render.s, /tmp/kernel.s
set -eu
cd "$(dirname "$0")/../cudaraytracer_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -mllvm -simplifycfg-sink-common=false --cuda-device-only -S render.hip \
    -o /tmp/render.s 2>&1 | grep -v hip-link || true
L=$(grep -n "^$1:" /tmp/render.s | cut -d: -f1)
awk -v L="$L" -v N="${2:-1500}" 'NR>=L && NR<=L+N' /tmp/render.s > /tmp/kernel.s
echo "kernel at line $L of /tmp/render.s; body in /tmp/kernel.s"
