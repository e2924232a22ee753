#!/bin/bash
# Build an experiment copy of libcatseg_hip.so with one source file recompiled under extra flags
# (e.g. -DSOME_MACRO, -fno-slp-vectorize), for same-box A/B runs through CATSEG_HIP_LIB.
# Usage: bash tools/build_exp.sh NAME FILE.hip "EXTRA FLAGS"   -> exp_so/libNAME.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FILE=$2; EXTRA=$3
make -C "$ROOT/cat-seg_amd/csrc" -j8 > /dev/null
mkdir -p "$ROOT/exp_so/$NAME"
OBJ="$ROOT/exp_so/$NAME/${FILE%.hip}.o"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -I"$ROOT/include" -I"$ROOT/cat-seg_amd/csrc" \
  -fno-honor-nans -Wno-unused-variable -Wno-unused-function -Wno-inline-asm $EXTRA -c "$ROOT/cat-seg_amd/csrc/$FILE" -o "$OBJ"
OBJS=$(ls "$ROOT"/build/csrc/*.o | grep -v "/${FILE%.hip}.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS "$OBJ" -o "$ROOT/exp_so/lib$NAME.so"
echo "$ROOT/exp_so/lib$NAME.so"
