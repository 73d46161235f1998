#!/bin/bash
# Build librt_hip.so with extra compile definitions into <out.so> (A/B experiments on the GPU box).
#   bash tools/build_variant_lib.sh <out.so> [-DNAME=VALUE ...]
set -eu
OUT=$(realpath -m "$1"); shift
cd "$(dirname "$0")/../cudaraytracer_amd/csrc"
T=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-slp-vectorize -mllvm -simplifycfg-sink-common=false "$@" -c render.hip -o $T/render.o
make -s -C . >/dev/null  # the host objects the library links (build/obj)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $T/render.o $(ls ../../build/obj/*.o | grep -v '/render.o$')
rm -rf $T
