// TEST INFRASTRUCTURE ONLY.  C entry points onto the reference's own HIP colour-
// conversion / layout launchers (src/rocjpeg_hip_kernels.cpp, compiled unmodified from
// /root/reference for gfx950 by oracle/build_ref.sh into oracle/_ref/).  Used on the
// GPU box to pin the oracle's CSC restatement and the product's fused output kernel
// against the reference kernels bit for bit.
#include <hip/hip_runtime.h>
#include "rocjpeg_hip_kernels.h"

#define S(x) reinterpret_cast<hipStream_t>(x)
extern "C" {
void ref_nv12_to_rgb(void *st, uint32_t w, uint32_t h, uint8_t *dst, uint32_t dp, const uint8_t *y, uint32_t yp,
                     const uint8_t *uv, uint32_t uvp) { ColorConvertNV12ToRGB(S(st), w, h, dst, dp, y, yp, uv, uvp); }
void ref_nv12_to_rgb_planar(void *st, uint32_t w, uint32_t h, uint8_t *r, uint8_t *g, uint8_t *b, uint32_t dp,
                            const uint8_t *y, uint32_t yp, const uint8_t *uv, uint32_t uvp) {
  ColorConvertNV12ToRGBPlanar(S(st), w, h, r, g, b, dp, y, yp, uv, uvp);
}
void ref_yuv444_to_rgb(void *st, uint32_t w, uint32_t h, uint8_t *dst, uint32_t dp, const uint8_t *base, uint32_t p,
                       uint32_t uoff, uint32_t voff) { ColorConvertYUV444ToRGB(S(st), w, h, dst, dp, base, p, uoff, voff); }
void ref_yuv440_to_rgb(void *st, uint32_t w, uint32_t h, uint8_t *dst, uint32_t dp, const uint8_t *base, uint32_t p,
                       uint32_t uoff, uint32_t voff) { ColorConvertYUV440ToRGB(S(st), w, h, dst, dp, base, p, uoff, voff); }
void ref_yuyv_to_rgb(void *st, uint32_t w, uint32_t h, uint8_t *dst, uint32_t dp, const uint8_t *src, uint32_t p) {
  ColorConvertYUYVToRGB(S(st), w, h, dst, dp, src, p);
}
void ref_yuv400_to_rgb(void *st, uint32_t w, uint32_t h, uint8_t *dst, uint32_t dp, const uint8_t *src, uint32_t p) {
  ColorConvertYUV400ToRGB(S(st), w, h, dst, dp, src, p);
}
void ref_yuv444_to_rgb_planar(void *st, uint32_t w, uint32_t h, uint8_t *r, uint8_t *g, uint8_t *b, uint32_t dp,
                              const uint8_t *base, uint32_t p, uint32_t uoff, uint32_t voff) {
  ColorConvertYUV444ToRGBPlanar(S(st), w, h, r, g, b, dp, base, p, uoff, voff);
}
void ref_yuv440_to_rgb_planar(void *st, uint32_t w, uint32_t h, uint8_t *r, uint8_t *g, uint8_t *b, uint32_t dp,
                              const uint8_t *base, uint32_t p, uint32_t uoff, uint32_t voff) {
  ColorConvertYUV440ToRGBPlanar(S(st), w, h, r, g, b, dp, base, p, uoff, voff);
}
void ref_yuyv_to_rgb_planar(void *st, uint32_t w, uint32_t h, uint8_t *r, uint8_t *g, uint8_t *b, uint32_t dp,
                            const uint8_t *src, uint32_t p) { ColorConvertYUYVToRGBPlanar(S(st), w, h, r, g, b, dp, src, p); }
void ref_yuv400_to_rgb_planar(void *st, uint32_t w, uint32_t h, uint8_t *r, uint8_t *g, uint8_t *b, uint32_t dp,
                              const uint8_t *src, uint32_t p) { ColorConvertYUV400ToRGBPlanar(S(st), w, h, r, g, b, dp, src, p); }
void ref_yuyv_extract_y(void *st, uint32_t w, uint32_t h, uint8_t *y, uint32_t yp, const uint8_t *src, uint32_t p) {
  ExtractYFromPackedYUYV(S(st), w, h, y, yp, src, p);
}
void ref_uv_to_planar(void *st, uint32_t w, uint32_t h, uint8_t *u, uint8_t *v, uint32_t dp, const uint8_t *uv, uint32_t p) {
  ConvertInterleavedUVToPlanarUV(S(st), w, h, u, v, dp, uv, p);
}
void ref_yuyv_to_planar(void *st, uint32_t w, uint32_t h, uint8_t *y, uint8_t *u, uint8_t *v, uint32_t yp, uint32_t cp,
                        const uint8_t *src, uint32_t p) { ConvertPackedYUYVToPlanarYUV(S(st), w, h, y, u, v, yp, cp, src, p); }
}
