#!/bin/bash
# Build A/B variants of librt_hip.so ON THE GPU BOX (no prebuilt libraries travel) into $AB_OUT (default
# /tmp/ablib): each argument is NAME=SOURCE[:SED_EXPR], SOURCE a render.hip path relative to the repo root,
# SED_EXPR an optional sed substitution applied to it first (a tools-side patch; the product source has no knobs).
#   bash tools/ab_variants_build.sh base=ab_src/render_precoop.hip coop=cudaraytracer_amd/csrc/render.hip \
#        'nocoop=cudaraytracer_amd/csrc/render.hip:s/PHILOX ? wl + P.lds_wave_words - CO_WORDS : nullptr/nullptr/'
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${AB_OUT:-/tmp/ablib}
mkdir -p "$OUT"
make -s -C "$ROOT/cudaraytracer_amd/csrc" >/dev/null  # host objects (build/obj)
for spec in "$@"; do
  name=${spec%%=*}; rest=${spec#*=}; src=${rest%%:*}; expr=""
  [ "$rest" != "$src" ] && expr=${rest#*:}
  T=$(mktemp -d)
  if [ -n "$expr" ]; then sed "$expr" "$ROOT/$src" > $T/render.hip; else cp "$ROOT/$src" $T/render.hip; fi
  cmp -s "$ROOT/$src" $T/render.hip && [ -n "$expr" ] && { echo "variant $name: patch matched nothing" >&2; exit 3; }
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-slp-vectorize \
    -mllvm -simplifycfg-sink-common=false -I"$ROOT/cudaraytracer_amd/csrc" -c $T/render.hip -o $T/render.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/$name.so" $T/render.o \
    $(ls "$ROOT"/build/obj/*.o | grep -v '/render.o$')
  rm -rf $T
  echo "built $OUT/$name.so"
done
