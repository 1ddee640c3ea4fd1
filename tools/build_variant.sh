#!/usr/bin/env bash
# Build librocjpeg_amd.so of another commit (default HEAD~1) as rocjpeg_amd/librocjpeg_amd_<name>.so
# for same-box A/B runs (RJ_LIB_PATH=...).  Development aid.
set -e
REV=${1:-HEAD~1}
NAME=${2:-prev}
ROOT=$(git rev-parse --show-toplevel)
TMP=$(mktemp -d /tmp/rjvar.XXXXXX)
git -C "$ROOT" archive "$REV" | tar -x -C "$TMP"
make -C "$TMP/rocjpeg_amd" -j8 >/dev/null
cp "$TMP/rocjpeg_amd/librocjpeg_amd.so" "$ROOT/rocjpeg_amd/librocjpeg_amd_$NAME.so"
rm -rf "$TMP"
echo "built $REV -> rocjpeg_amd/librocjpeg_amd_$NAME.so"
