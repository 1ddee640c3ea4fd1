#!/usr/bin/env bash
# Builds the reference's own sources (read in place from /root/reference, never copied)
# into oracle/_ref/ -- TEST INFRASTRUCTURE ONLY.  Only two translation units of the
# reference are self-contained enough to build here:
#   src/rocjpeg_parser.cpp      (std C++ only)          -> _ref/librefparser.so  (g++)
#   src/rocjpeg_hip_kernels.cpp (HIP only, for gfx950)  -> _ref/librefcsc.so     (hipcc)
# The VCN decode core (src/rocjpeg_vaapi_decoder.cpp) needs libva/va.h, absent from this
# image: it is unbuildable here and is not attempted.
set -euo pipefail
REF=${REFERENCE_ROOT:-/root/reference}
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT="$HERE/_ref"
if [ ! -f "$REF/src/rocjpeg_parser.cpp" ]; then
  echo "reference not present at $REF: keeping prebuilt oracle/_ref (if any)"; exit 0
fi
mkdir -p "$OUT"
g++ -O2 -std=c++17 -fPIC -shared -w -I"$REF/src" -o "$OUT/librefparser.so" \
    "$REF/src/rocjpeg_parser.cpp" "$HERE/ref_shims/ref_parser_shim.cpp"
if command -v hipcc >/dev/null 2>&1; then
  hipcc --offload-arch=gfx950 -O3 -fPIC -shared -w -I"$REF/src" -o "$OUT/librefcsc.so" \
      "$REF/src/rocjpeg_hip_kernels.cpp" "$HERE/ref_shims/ref_csc_shim.cpp"
fi
echo "built: $(ls "$OUT")"
