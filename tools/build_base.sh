#!/bin/bash
# Build libcordagpu.so from a git revision (default HEAD) into tools/variants/<name>.so, for A/B
# runs against the working tree (tools/ab.sh).  usage: bash tools/build_base.sh [rev] [name]
set -e
REV=${1:-HEAD}
NAME=${2:-base}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" corda_amd/csrc include | tar -x -C "$TMP"
make -s -j8 -C "$TMP/corda_amd/csrc" >/dev/null
mkdir -p "$ROOT/tools/variants"
cp "$TMP/corda_amd/libcordagpu.so" "$ROOT/tools/variants/$NAME.so"
rm -rf "$TMP"
echo "tools/variants/$NAME.so"
