#!/usr/bin/env bash
# Build the working tree's library with K2 phase stamps (RJ_EXP_STAMPS) as
# rocjpeg_amd/librocjpeg_amd_stamps.so (run with RJ_LIB_PATH=... RJ_DEBUG_STAMPS=1).  Development aid.
set -e
ROOT=$(git rev-parse --show-toplevel)
TMP=$(mktemp -d /tmp/rjstamps.XXXXXX)
cp -r "$ROOT/rocjpeg_amd" "$ROOT/include" "$TMP/"
rm -f "$TMP"/rocjpeg_amd/csrc/*.o "$TMP"/rocjpeg_amd/*.so
make -C "$TMP/rocjpeg_amd" -j8 EXTRA=-DRJ_EXP_STAMPS >/dev/null
cp "$TMP/rocjpeg_amd/librocjpeg_amd.so" "$ROOT/rocjpeg_amd/librocjpeg_amd_stamps.so"
rm -rf "$TMP"
echo "built rocjpeg_amd/librocjpeg_amd_stamps.so"
