#!/bin/bash
# Export the library sources of a git revision, optionally with a patch applied, into ab_src/tree_<name>/ (git-ignored,
# but carried to the GPU box by gpurun, whose snapshot has no .git): tools/ab_variants_build.sh builds NAME=@<name>
# from it.  Run it where the repository's history is (the A/B scripts call it when the tree is missing).
#   bash tools/ab_prepare.sh <name> <rev> [patch relative to the repo root]
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; rev=$2; patch=${3:-}
out=$ROOT/ab_src/tree_$name
if ! git -C "$ROOT" rev-parse --verify -q "$rev^{commit}" > /dev/null; then
  echo "ab_prepare: revision $rev not found (no git history here? run this script where the repository is)" >&2
  exit 2
fi
rm -rf "$out"; mkdir -p "$out"
git -C "$ROOT" archive "$rev" cudaraytracer_amd include tests | tar -x -C "$out"
if [ -n "$patch" ]; then patch -d "$out" -p1 --forward --quiet < "$ROOT/$patch" || { echo "ab_prepare: $patch does not apply to $rev" >&2; exit 3; }; grep -q . "$ROOT/$patch" || exit 3; fi
echo "ab_prepare: $out = $rev${patch:+ + $patch}"
