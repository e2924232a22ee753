#!/bin/bash
# Build the library of a git revision (default HEAD) to cat-seg_amd/cat_seg/libcatseg_hip_ref.so
# for a same-box A/B with tools/_ab.sh.  Usage: bash tools/build_ref_so.sh [REV]
set -e
REV=${1:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/catseg_ref.XXXX)
git -C "$R" worktree add -q "$T/tree" "$REV"
make -C "$T/tree/cat-seg_amd/csrc" -j8 BUILD="$T/build" OUT="$R/cat-seg_amd/cat_seg/libcatseg_hip_ref.so" > "$T/make.log" 2>&1 || { tail -20 "$T/make.log"; exit 1; }
git -C "$R" worktree remove --force "$T/tree"
rm -rf "$T"
