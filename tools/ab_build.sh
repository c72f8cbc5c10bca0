#!/bin/bash
# Build libpano.so of git revision $1 into tools/ab/libpano_$1.so (A/B timing against the
# working tree in ONE gpurun call: PANO_LIB=tools/ab/libpano_<rev>.so python bench.py ...).
set -e
REV=${1:?revision}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" vfx_image_stitching_amd/csrc include | tar -x -C "$TMP"
mkdir -p "$ROOT/tools/ab"
make -C "$TMP/vfx_image_stitching_amd/csrc" -j8 OUT="$ROOT/tools/ab/libpano_$REV.so" >/dev/null
rm -rf "$TMP"
echo "$ROOT/tools/ab/libpano_$REV.so"
