#!/usr/bin/env bash
# Build the working tree's library with extra compile flags as rocjpeg_amd/librocjpeg_amd_<name>.so
# (A/B runs: RJ_LIB_PATH=$PWD/rocjpeg_amd/librocjpeg_amd_<name>.so).  Development aid.
#   tools/build_flags.sh <name> "<flags>"
set -e
ROOT=$(git rev-parse --show-toplevel)
TMP=$(mktemp -d /tmp/rjflags.XXXXXX)
mkdir -p "$TMP/rocjpeg_amd"
cp -r "$ROOT/rocjpeg_amd/csrc" "$ROOT/rocjpeg_amd/Makefile" "$TMP/rocjpeg_amd/"
cp -r "$ROOT/include" "$TMP/"
make -C "$TMP/rocjpeg_amd" -j8 EXTRA="$2" librocjpeg_amd.so >/dev/null
cp "$TMP/rocjpeg_amd/librocjpeg_amd.so" "$ROOT/rocjpeg_amd/librocjpeg_amd_$1.so"
rm -rf "$TMP"
echo "built rocjpeg_amd/librocjpeg_amd_$1.so ($2)"
