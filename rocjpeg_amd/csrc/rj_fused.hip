// rj_fused.hip -- K2 fused output kernel: dequant + ISLOW IDCT + nearest chroma upsample +
// YUV->RGB (or planar layouts) straight from the coefficient blocks to the caller's buffers.
//
// One workgroup (256 threads = 4 waves) per strip: one MCU row x 256 pixels (16 MCUs at
// 4:2:0).  HBM traffic per strip = its coefficient blocks (read once, contiguous: the MCU-major
// layout K1 writes) + its output bytes (written once, whole 16-B chunks per lane).
// LDS per workgroup (4:2:0): 12 KB coefficients aliased by the sample tiles + 24 KB pass-1
// workspace + quant tables ~= 37 KB -> 4 workgroups per CU.
//
// Same integer IDCT (rj_math.h islow_1d) and the same CSC (rj_math.h csc_pixel) as the general
// path, so both paths are bit-identical; eligibility (no ROI, canonical sampling geometry,
// copy channels with pitch == width) is decided on the host (rj_decoder.cpp).
#include <hip/hip_runtime.h>

#include "rj_device.h"
#include "rj_kernels.h"
#include "rj_math.h"

namespace rj {

#define RJ_STRIP_PX 256
#define RJ_MAX_STRIP_BLK 128

__global__ __launch_bounds__(256) void k_fused(const RjImageDev *__restrict__ imgs, int nimg,
                                               const uint32_t *__restrict__ strip_prefix,
                                               const int16_t *__restrict__ coefs,
                                               const RjTableSet *__restrict__ tabsets) {
  __shared__ __attribute__((aligned(16))) int16_t s_coef[RJ_MAX_STRIP_BLK * 64];  // later: sample tiles
  __shared__ __attribute__((aligned(16))) int32_t s_ws[RJ_MAX_STRIP_BLK * 64];
  __shared__ int32_t s_q[3][64];
  __shared__ uint32_t s_tile_off[3], s_tile_w[3];

  const uint32_t tid = threadIdx.x;
  const uint32_t sg = blockIdx.x;
  const int i = [&] {
    int lo = 0, hi = nimg - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (strip_prefix[mid] <= sg) lo = mid;
      else hi = mid - 1;
    }
    return lo;
  }();
  const RjImageDev &im = imgs[i];
  const uint32_t hmax = im.hmax, vmax = im.vmax;
  const uint32_t mcu_w = 8 * hmax, mcu_h = 8 * vmax;
  const uint32_t S = RJ_STRIP_PX / mcu_w;               // MCUs per strip
  const uint32_t strips_x = (im.mcux + S - 1) / S;
  const uint32_t local = sg - strip_prefix[i];
  const uint32_t my = local / strips_x;
  const uint32_t mx0 = (local - my * strips_x) * S;
  const uint32_t nm = min(S, im.mcux - mx0);           // MCUs in this strip
  const uint32_t nblk = im.nblk_mcu;
  const uint32_t nb = nm * nblk;                        // blocks in this strip
  const uint32_t ncomp = im.interleaved ? im.ncomp : 1;

  // ---- quant tables + tile geometry ----
  const RjTableSet *ts = tabsets + im.tabset;
  for (uint32_t k = tid; k < ncomp * 64; k += 256) s_q[k >> 6][k & 63] = ts->q[im.comp_tq[k >> 6] & 3][k & 63];
  if (tid == 0) {
    uint32_t off = 0;
    for (uint32_t c = 0; c < ncomp; c++) {
      const uint32_t hc = im.interleaved ? im.comp_h[c] : 1, vc = im.interleaved ? im.comp_v[c] : 1;
      s_tile_w[c] = S * hc * 8;
      s_tile_off[c] = off;
      off += S * hc * 8 * vc * 8;
    }
  }
  // ---- phase A: coefficient blocks -> LDS (contiguous, 16 B per lane) ----
  {
    const uint4 *src = reinterpret_cast<const uint4 *>(coefs + (im.coef_off + (uint64_t(my) * im.mcux + mx0) * nblk) * 64u);
    uint4 *dst = reinterpret_cast<uint4 *>(s_coef);
    const uint32_t n16 = nb * 8;
    for (uint32_t k = tid; k < n16; k += 256) dst[k] = src[k];
  }
  __syncthreads();
  // ---- phase B1: column pass (block, column) -> s_ws ----
  for (uint32_t t = tid; t < nb * 8; t += 256) {
    const uint32_t blk = t >> 3, col = t & 7;
    const uint32_t c = im.interleaved ? im.blk_comp[blk % nblk] : 0;
    const int16_t *in = s_coef + blk * 64 + col;
    const int32_t *q = s_q[c] + col;
    int32_t o[8];
    islow_1d(in[0] * q[0], in[8] * q[8], in[16] * q[16], in[24] * q[24], in[32] * q[32], in[40] * q[40],
             in[48] * q[48], in[56] * q[56], o);
    int32_t *w = s_ws + blk * 64 + col;
#pragma unroll
    for (int r = 0; r < 8; r++) w[r * 8] = (o[r] + 1024) >> 11;
  }
  __syncthreads();
  // ---- phase B2: row pass (block, row) -> sample tiles (aliasing s_coef) ----
  uint8_t *tiles = reinterpret_cast<uint8_t *>(s_coef);
  for (uint32_t t = tid; t < nb * 8; t += 256) {
    const uint32_t blk = t >> 3, row = t & 7;
    const uint32_t mcu = blk / nblk, b = blk - mcu * nblk;
    const uint32_t c = im.interleaved ? im.blk_comp[b] : 0;
    const uint32_t hc = im.interleaved ? im.comp_h[c] : 1;
    const uint32_t dx = im.interleaved ? im.blk_dx[b] : 0, dy = im.interleaved ? im.blk_dy[b] : 0;
    const int32_t *w = s_ws + blk * 64 + row * 8;
    int32_t o[8];
    islow_1d(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], o);
    uint2 pk;
    pk.x = islow_range_limit((o[0] + (1 << 17)) >> 18) | (islow_range_limit((o[1] + (1 << 17)) >> 18) << 8) |
           (islow_range_limit((o[2] + (1 << 17)) >> 18) << 16) | (islow_range_limit((o[3] + (1 << 17)) >> 18) << 24);
    pk.y = islow_range_limit((o[4] + (1 << 17)) >> 18) | (islow_range_limit((o[5] + (1 << 17)) >> 18) << 8) |
           (islow_range_limit((o[6] + (1 << 17)) >> 18) << 16) | (islow_range_limit((o[7] + (1 << 17)) >> 18) << 24);
    const uint32_t tx = (mcu * hc + dx) * 8, ty = dy * 8 + row;
    *reinterpret_cast<uint2 *>(tiles + s_tile_off[c] + ty * s_tile_w[c] + tx) = pk;
  }
  __syncthreads();

  // ---- phase C: output ----
  const uint32_t strip_w = nm * mcu_w;                  // pixels in this strip
  const uint32_t px0 = mx0 * mcu_w, py0 = my * mcu_h;
  const uint32_t W = im.width, H = im.height;
  const uint32_t fmt = im.fmt;
  const uint8_t *ty0 = tiles + s_tile_off[0];
  const uint32_t tw0 = s_tile_w[0];
  // chroma sampling ratios (canonical geometries only: power-of-two ratios)
  const uint32_t hs1 = (im.ncomp == 3) ? (hmax / im.comp_h[1] == 2 ? 1u : 0u) : 0u;
  const uint32_t vs1 = (im.ncomp == 3) ? (vmax / im.comp_v[1] == 2 ? 1u : 0u) : 0u;

  if (fmt >= 1 && fmt <= 4) {
    // luma-resolution pass: 16-pixel chunks
    const uint32_t chunks_x = (strip_w + 15) / 16;
    const uint32_t nchunks = chunks_x * mcu_h;
    for (uint32_t k = tid; k < nchunks; k += 256) {
      const uint32_t y = k / chunks_x, xc = (k - y * chunks_x) * 16;
      const uint32_t py = py0 + y;
      if (py >= H) continue;
      const uint32_t px = px0 + xc;
      if (px >= W) continue;
      const uint32_t n = min(16u, min(strip_w - xc, W - px));
      const uint8_t *yrow = ty0 + y * tw0 + xc;
      if (fmt == 3 || fmt == 4) {
        uint32_t w[12];  // 16 RGB pixels packed little-endian, constant-indexed (stays in VGPRs)
#pragma unroll
        for (int q = 0; q < 12; q++) w[q] = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) {
          uint32_t p3;
          if (im.ncomp == 3) {
            const uint32_t cx = (xc + j) >> hs1;
            p3 = csc_pixel_packed(yrow[j], tiles[s_tile_off[1] + (y >> vs1) * s_tile_w[1] + cx],
                                  tiles[s_tile_off[2] + (y >> vs1) * s_tile_w[2] + cx]);
          } else {
            p3 = uint32_t(yrow[j]) * 0x010101u;
          }
#pragma unroll
          for (int e = 0; e < 3; e++) w[(3 * j + e) >> 2] |= ((p3 >> (8 * e)) & 255u) << (8 * ((3 * j + e) & 3));
        }
        if (fmt == 3) {
          uint8_t *d = im.dst[0] + uint64_t(py) * im.dst_pitch[0] + uint64_t(px) * 3;
          if (n == 16 && ((reinterpret_cast<uintptr_t>(d) & 15) == 0)) {
            uint4 *d4 = reinterpret_cast<uint4 *>(d);
            d4[0] = make_uint4(w[0], w[1], w[2], w[3]);
            d4[1] = make_uint4(w[4], w[5], w[6], w[7]);
            d4[2] = make_uint4(w[8], w[9], w[10], w[11]);
          } else {
#pragma unroll
            for (int j = 0; j < 48; j++)
              if (uint32_t(j) < 3 * n) d[j] = uint8_t(w[j >> 2] >> (8 * (j & 3)));
          }
        } else {
#pragma unroll
          for (int p = 0; p < 3; p++) {
            uint32_t pl[4] = {0, 0, 0, 0};
#pragma unroll
            for (int j = 0; j < 16; j++) {
              const int b = 3 * j + p;
              pl[j >> 2] |= ((w[b >> 2] >> (8 * (b & 3))) & 255u) << (8 * (j & 3));
            }
            uint8_t *d = im.dst[p] + uint64_t(py) * im.dst_pitch[0] + px;
            if (n == 16 && ((reinterpret_cast<uintptr_t>(d) & 15) == 0)) {
              *reinterpret_cast<uint4 *>(d) = make_uint4(pl[0], pl[1], pl[2], pl[3]);
            } else {
#pragma unroll
              for (int j = 0; j < 16; j++)
                if (uint32_t(j) < n) d[j] = uint8_t(pl[j >> 2] >> (8 * (j & 3)));
            }
          }
        }
      } else {  // Y plane (OUTPUT_Y and the luma of YUV_PLANAR)
        uint8_t *d = im.dst[0] + uint64_t(py) * im.dst_pitch[0] + px;
        if (n == 16 && ((reinterpret_cast<uintptr_t>(d) & 15) == 0) && ((reinterpret_cast<uintptr_t>(yrow) & 15) == 0)) {
          *reinterpret_cast<uint4 *>(d) = *reinterpret_cast<const uint4 *>(yrow);
        } else {
          for (uint32_t j = 0; j < n; j++) d[j] = yrow[j];
        }
      }
    }
  }
  if (fmt == 1 && im.ncomp == 3) {  // chroma planes of YUV_PLANAR at native resolution
#pragma unroll
    for (int c = 1; c < 3; c++) {
      const uint32_t hc = im.comp_h[c], vc = im.comp_v[c];
      const uint32_t cw = nm * hc * 8, ch = vc * 8;
      const uint32_t cx0 = mx0 * hc * 8, cy0 = my * vc * 8;
      const uint32_t cW = (hs1 ? (W >> 1) : W), cH = (vs1 ? (H >> 1) : H);
      const uint32_t chunks_x = (cw + 15) / 16;
      for (uint32_t k = tid; k < chunks_x * ch; k += 256) {
        const uint32_t y = k / chunks_x, xc = (k - y * chunks_x) * 16;
        const uint32_t py = cy0 + y, px = cx0 + xc;
        if (py >= cH || px >= cW) continue;
        const uint32_t n = min(16u, min(cw - xc, cW - px));
        const uint8_t *srow = tiles + s_tile_off[c] + y * s_tile_w[c] + xc;
        uint8_t *d = im.dst[c] + uint64_t(py) * im.dst_pitch[1] + px;  // U and V share pitch[1] (host-checked)
        if (n == 16 && ((reinterpret_cast<uintptr_t>(d) & 15) == 0)) {
          *reinterpret_cast<uint4 *>(d) = *reinterpret_cast<const uint4 *>(srow);
        } else {
          for (uint32_t j = 0; j < n; j++) d[j] = srow[j];
        }
      }
    }
  }
}

hipError_t LaunchFusedOutput(hipStream_t st, const RjImageDev *imgs, int nimg, const uint32_t *strip_prefix,
                             uint32_t nstrips, const int16_t *coefs, const RjTableSet *tabsets) {
  if (nstrips == 0) return hipSuccess;
  hipLaunchKernelGGL(k_fused, dim3(nstrips), dim3(256), 0, st, imgs, nimg, strip_prefix, coefs, tabsets);
  return hipGetLastError();
}

}  // namespace rj
