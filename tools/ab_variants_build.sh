#!/bin/bash
# Build A/B variants of librt_hip.so ON THE GPU BOX (no prebuilt libraries travel) into $AB_OUT (default /tmp/ablib).
# Each argument is one of
#   NAME=SOURCE[:SED_EXPR]  SOURCE a render.hip path relative to the repo root, SED_EXPR an optional sed substitution
#                           applied to it first (a tools-side patch; the product source has no knobs for it), linked
#                           with the current tree's host objects;
#   NAME=@TREE              the whole library of a revision exported by tools/ab_prepare.sh into ab_src/tree_TREE.
#   bash tools/ab_variants_build.sh 'nothr=cudaraytracer_amd/csrc/render.hip:s/thr = thr > deferred + 1u ? thr - deferred : 1u;/(void)deferred;/'
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${AB_OUT:-/tmp/ablib}
mkdir -p "$OUT"
make -s -C "$ROOT/cudaraytracer_amd/csrc" >/dev/null  # host objects (build/obj)
for spec in "$@"; do
  name=${spec%%=*}; rest=${spec#*=}
  if [ "${rest#@}" != "$rest" ]; then
    tree=$ROOT/ab_src/tree_${rest#@}
    [ -d "$tree" ] || { echo "variant $name: $tree missing (tools/ab_prepare.sh ${rest#@} <rev>)" >&2; exit 3; }
    make -s -C "$tree/cudaraytracer_amd/csrc" >/dev/null
    cp "$tree/cudaraytracer_amd/librt_hip.so" "$OUT/$name.so"
    echo "built $OUT/$name.so from $tree"
    continue
  fi
  src=${rest%%:*}; expr=""
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
