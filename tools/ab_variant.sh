#!/bin/bash
# Build the working tree's libpano.so with extra compiler flags into tools/ab/libpano_<name>.so
# (A/B probes in one gpurun call: PANO_LIB=tools/ab/libpano_<name>.so ...).
set -e
NAME=${1:?name}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
cp -r "$ROOT/vfx_image_stitching_amd/csrc" "$TMP/csrc"; mkdir -p "$TMP/include" && cp "$ROOT/include/pano.h" "$TMP/include/"
mkdir -p "$TMP/x" && mv "$TMP/csrc" "$TMP/x/csrc" && rm -rf "$TMP/x/csrc/build"
mkdir -p "$ROOT/tools/ab"
make -C "$TMP/x/csrc" -j8 EXTRA="$*" OUT="$ROOT/tools/ab/libpano_$NAME.so" >/dev/null
rm -rf "$TMP"
echo "$ROOT/tools/ab/libpano_$NAME.so"
