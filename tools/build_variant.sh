#!/bin/bash
# Build libcordagpu.so from the working tree with extra compile flags into tools/variants/<name>.so,
# for A/B runs (tools/ab.sh).  usage: bash tools/build_variant.sh <name> "-DED_FINISH_K=32 ..."
set -e
NAME=$1
EXTRA=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
mkdir -p "$TMP/corda_amd" && cp -r "$ROOT/corda_amd/csrc" "$TMP/corda_amd/" && cp -r "$ROOT/include" "$TMP/"
rm -rf "$TMP/corda_amd/csrc/build"
make -s -j8 -C "$TMP/corda_amd/csrc" HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-result -Wno-unused-value $EXTRA" >/dev/null
mkdir -p "$ROOT/tools/variants"
cp "$TMP/corda_amd/libcordagpu.so" "$ROOT/tools/variants/$NAME.so"
rm -rf "$TMP"
echo "tools/variants/$NAME.so"
