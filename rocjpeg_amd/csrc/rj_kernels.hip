// rj_kernels.hip -- the JPEG decode hot path for MI355X (gfx950, wave64).
//
// Replaces the VCN fixed-function decode of the reference (src/rocjpeg_vaapi_decoder.cpp:
// 574-692) and rewrites its post-processing kernels (src/rocjpeg_hip_kernels.cpp).
//
//   K0 k_destuff      one wavefront per 2-KB block of entropy-coded bytes (output offsets from
//                     the host parser): FF00/fill removal by per-lane keep masks + wave prefix
//                     sum, compacted stores.
//   K1 k_entropy      (rj_entropy.hip) Huffman decode, one lane per interval chunk, with
//                     self-synchronising speculative chunks for long intervals.
//   K2 k_rows         (rj_fused.hip) one wave per MCU row: entry stream -> LDS blocks ->
//                     dequant + ISLOW IDCT -> fused output (upsample + CSC / layout) or
//                     MCU-padded component planes (general path).
//   K2b k_output      every output format / ROI semantic of rocjpeg_decoder.cpp:143-180,
//                     colour conversion identical to rocjpeg_hip_kernels.cpp:1431-1443.
#include <hip/hip_runtime.h>

#include "rj_device.h"
#include "rj_kernels.h"
#include "rj_math.h"

namespace rj {

// ---------------------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------------------
// exclusive prefix sum over the wave (DPP scan, no LDS round trips); total: the wave's sum
__device__ __forceinline__ uint32_t wave_exclusive_scan(uint32_t v, uint32_t &total) {
  const uint32_t x = uint32_t(wave_scan(int(v)));
  total = __builtin_amdgcn_readlane(x, 63);
  return x - v;
}

// ---------------------------------------------------------------------------------------
// K0: destuff.  Within an interval's raw range the host guarantees only data bytes,
// FF 00 pairs and FF fill runs in front of an FF 00 occur.  Byte i is dropped when
// (b[i] == 00 && b[i-1] == FF) or (b[i] == FF && b[i+1] == FF).
// kLds: the block's output is assembled in LDS (a chunk with an FF byte as LDS byte writes at
// its compacted offsets) and leaves as aligned dword stores, bytes only at the two ends; without
// it, such a chunk's bytes were four global byte stores per lane (~2/3 of 256-B chunks hold an
// FF byte).
// ---------------------------------------------------------------------------------------
template <bool kLds>
__global__ __launch_bounds__(64) void k_destuff(const RjImageDev *__restrict__ imgs, int nimg,
                                                uint8_t *__restrict__ destuffed, const uint32_t *__restrict__ ds_map) {
  static_assert(RJ_DS_BLOCK % 256u == 0 && RJ_DS_BLOCK <= 4096u, "256-B chunks, all loads issued up front");
  constexpr int kIt = RJ_DS_BLOCK / 256;
  // LDS byte m + t holds output byte t (m: the output's misalignment, so LDS dword k is the
  // output's aligned dword k)
  __shared__ uint32_t s_out[kLds ? RJ_DS_BLOCK / 4 + 2 : 1];
  uint8_t *const sb = reinterpret_cast<uint8_t *>(s_out);
  const uint32_t g = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  // the block's image: between the owners of blocks 64 (g / 64) and 64 (g / 64 + 1) (the host's
  // map), usually one or two images apart -- a search over all images was ten dependent loads
  // in front of every block's data loads, which made K0 latency-bound
  int lo = 0, hi = nimg - 1;
  if (ds_map != nullptr) {
    lo = int(ds_map[g >> 6]);
    hi = int(ds_map[(g >> 6) + 1]);
  }
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (imgs[mid].ds_prefix <= g) lo = mid;
    else hi = mid - 1;
  }
  const int i = __builtin_amdgcn_readfirstlane(lo);
  const RjImageDev &im = imgs[i];
  const RjDsBlock blk = gp(im.ds)[g - im.ds_prefix];
  const RJ_GLOBAL uint8_t *src = gp(im.ecs + blk.src_off);
  uint8_t *dst = destuffed + im.destuff_off + blk.dst_off;
  const bool first = (blk.len >> 31) != 0;  // first block of its interval
  const uint32_t len = blk.len & 0x7FFFFFFFu;
  const bool last = blk.zero_end != 0;
  // every load of the block is issued up front (one memory latency per block, not per chunk):
  // lane l of chunk c takes bytes [256c + 4l, +4) from two aligned dwords (alignbyte), the
  // dword index clamped into the block (the ECS buffers carry >= 16 B of slack)
  const uint32_t mis = uint32_t(reinterpret_cast<uintptr_t>(src)) & 3u;
  const RJ_GLOBAL uint32_t *A = reinterpret_cast<const RJ_GLOBAL uint32_t *>(src - mis);
  const uint32_t last_dw = len ? (len - 1 + mis) >> 2 : 0u;
  uint32_t w[kIt];
#pragma unroll
  for (int c = 0; c < kIt; c++) {
    const uint32_t q = min(uint32_t(c) * 64u + lane, last_dw);
    w[c] = __builtin_amdgcn_alignbyte(A[q + 1], A[q], mis);
  }
  const uint32_t before = first ? 0u : uint32_t(src[-1]);       // byte in front of the block
  const uint32_t after = last ? 0x100u : uint32_t(src[len]);     // byte behind it (0x100: none)
  uint32_t out = 0;
  uint32_t prev_byte = before;  // byte in front of the current chunk
  const uint32_t m0 = uint32_t(reinterpret_cast<uintptr_t>(dst)) & 3u;
#pragma unroll
  for (int c = 0; c < kIt; c++) {
    const uint32_t base = uint32_t(c) * 256u;
    if (base >= len) break;  // wave-uniform
    // fast path: a whole chunk with no FF byte (and no FF in front of it) keeps every byte --
    // aligned dword stores: dword j of the output gets lane j-1's top bytes and lane j's low ones
    {
      const uint32_t t = ~w[c];
      const bool ff = ((t - 0x01010101u) & ~t & 0x80808080u) != 0;  // some byte == 0xFF
      if (base + 256u <= len && prev_byte != 0xFFu && __builtin_amdgcn_ballot_w64(ff) == 0) {
        const uint32_t wc = w[c];
        if constexpr (kLds) {
          const uint32_t pos = m0 + out, a = pos & 3u, k0 = pos >> 2;
          if (a == 0) {
            s_out[k0 + lane] = wc;
          } else {
            const uint32_t e = __builtin_amdgcn_alignbyte(wc, wave_prev(wc), 4u - a);
            if (lane > 0) s_out[k0 + lane] = e;
            else s_out[k0] = (s_out[k0] & ((1u << (8 * a)) - 1u)) | (wc << (8 * a));  // after the bytes before
            if (lane == 63) s_out[k0 + 64] = wc >> (8 * (4 - a));
          }
          out += 256u;
          prev_byte = __builtin_amdgcn_readlane(wc, 63) >> 24;
          continue;
        }
        const uint32_t m = uint32_t(reinterpret_cast<uintptr_t>(dst) + out) & 3u;  // wave-uniform
        uint8_t *D = dst + out - m;  // 4-B aligned
        if (m == 0) {
          *gp(reinterpret_cast<uint32_t *>(D) + lane) = wc;
        } else {
          const uint32_t e = __builtin_amdgcn_alignbyte(wc, wave_prev(wc), 4u - m);
          if (lane > 0) *gp(reinterpret_cast<uint32_t *>(D) + lane) = e;
          if (lane == 0)
            for (uint32_t k = 0; k < 4u - m; k++) gp(D)[m + k] = uint8_t(wc >> (8 * k));
          if (lane == 63)
            for (uint32_t k = 4u - m; k < 4u; k++) gp(D)[256u + k - (4u - m)] = uint8_t(wc >> (8 * k));
        }
        out += 256u;
        prev_byte = __builtin_amdgcn_readlane(wc, 63) >> 24;
        continue;
      }
    }
    const uint32_t p = base + 4 * lane;
    uint32_t b[4];
#pragma unroll
    for (int k = 0; k < 4; k++) b[k] = (p + k < len) ? (w[c] >> (8 * k)) & 255u : 0x100u;  // 0x100 = past the end
    // the byte after this chunk: the next chunk's first byte, or the one behind the block
    uint32_t nb_next = after;
    if (c + 1 < kIt && base + 256 < len) nb_next = __builtin_amdgcn_readfirstlane(w[c + 1]) & 255u;
    uint32_t prev = wave_prev(b[3]);
    if (lane == 0) prev = prev_byte;
    uint32_t next = wave_next(b[0]);
    if (lane == 63) next = nb_next;
    uint32_t keep = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t pv = k == 0 ? prev : b[k - 1];
      uint32_t nx = k == 3 ? next : b[k + 1];
      if (p + k + 1 == len) nx = after;  // the block's last byte
      const bool drop = b[k] == 0x100u || (b[k] == 0x00u && pv == 0xFFu) || (b[k] == 0xFFu && nx == 0xFFu);
      keep |= (drop ? 0u : 1u) << k;
    }
    uint32_t total;
    uint32_t o = wave_exclusive_scan(__popc(keep), total) + out;
    if constexpr (kLds) {
      o += m0;
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (keep & (1u << k)) sb[o++] = uint8_t(b[k]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (keep & (1u << k)) gp(dst)[o++] = uint8_t(b[k]);
    }
    out += total;
    prev_byte = __builtin_amdgcn_readlane(b[3], 63);
  }
  if constexpr (kLds) {
    // LDS -> the output: aligned dwords [k_lo, k_hi), the bytes of a partial dword at either end
    // (the head's bytes before m0 belong to the block in front)
    __syncthreads();
    const uint32_t end = m0 + out, k_lo = (m0 + 3u) >> 2, k_hi = end >> 2;
    uint32_t *const D = reinterpret_cast<uint32_t *>(dst - m0);
    for (uint32_t k = k_lo + lane; k < k_hi; k += 64) gp(D)[k] = s_out[k];
    const uint32_t hb = lane, tb = 4u * max(k_hi, k_lo) + (lane - 4u);
    if (lane < 4 && hb >= m0 && hb < min(4u * k_lo, end)) gp(dst - m0)[hb] = sb[hb];
    if (lane >= 4 && lane < 8 && tb < end) gp(dst - m0)[tb] = sb[tb];
  }
  // last block: zero the interval's slack after the data (>= 16 B, rj_stream.cpp BuildPlan):
  // K1 reads whole 16-B chunks and must see zero bits past the end, as libjpeg inserts
  if (last) {
    uint8_t *base = destuffed + im.destuff_off;
    for (uint32_t q = blk.dst_off + out + lane; q < blk.zero_end; q += 64) gp(base)[q] = 0;
  }
}

hipError_t LaunchDestuff(hipStream_t st, const RjImageDev *imgs, int nimg, uint32_t nblocks, uint8_t *destuffed,
                         const uint32_t *ds_map, bool lds) {
  if (nblocks == 0) return hipSuccess;
  if (lds) hipLaunchKernelGGL(k_destuff<true>, dim3(nblocks), dim3(64), 0, st, imgs, nimg, destuffed, ds_map);
  else hipLaunchKernelGGL(k_destuff<false>, dim3(nblocks), dim3(64), 0, st, imgs, nimg, destuffed, ds_map);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// K2b: general output stage over the VCN-surface model (see oracle oj_decode).
// ---------------------------------------------------------------------------------------
struct PlaneView {
  const uint8_t *base;
  const RjImageDev *im;
  __device__ __forceinline__ uint8_t px(int c, int64_t r, int64_t x) const {
    const int64_t rows = im->plane_rows[c], pitch = im->plane_pitch[c];
    r = r < 0 ? 0 : (r >= rows ? rows - 1 : r);
    x = x < 0 ? 0 : (x >= pitch ? pitch - 1 : x);
    return base[im->plane_off[c] + uint64_t(r) * uint64_t(pitch) + uint64_t(x)];
  }
  // byte b of row r of surface plane sp (0 = luma / packed YUYV, 1 = chroma) for channel chan
  __device__ __forceinline__ uint8_t surf(int sp, int chan, int64_t r, int64_t b) const {
    if (im->css == 2 && sp == 0) {  // YUYV
      const int64_t q = b >> 2;
      switch (b & 3) {
        case 0: return px(0, r, 2 * q);
        case 1: return px(1, r, q);
        case 2: return px(0, r, 2 * q + 1);
        default: return px(2, r, q);
      }
    }
    if (im->css == 3 && sp == 1) return (b & 1) ? px(2, r, b >> 1) : px(1, r, b >> 1);  // NV12 UV
    return px(chan, r, b);
  }
  __device__ __forceinline__ void rgb(int64_t y, int64_t x, uint8_t out[3]) const {
    const int64_t top = im->top, left = im->left;
    const uint8_t Y = px(0, top + y, left + x);
    uint8_t U = 128, V = 128;
    switch (im->css) {
      case 0:  // 4:4:4 -- luma ROI offset applied twice (rocjpeg_decoder.cpp:464-467)
        U = px(1, 2 * top + y, 2 * left + x);
        V = px(2, 2 * top + y, 2 * left + x);
        break;
      case 1:  // 4:4:0 -- chroma ROI offset commented out (rocjpeg_decoder.cpp:470)
        U = px(1, top + (y >> 1), left + x);
        V = px(2, top + (y >> 1), left + x);
        break;
      case 2: {  // YUYV read from byte 2*left
        const int64_t b = 2 * left + 4 * (x >> 1);
        U = surf(0, 0, top + y, b + 1);
        V = surf(0, 0, top + y, b + 3);
        break;
      }
      case 3: {  // NV12: UV + (top>>1)*pitch + left
        const int64_t b = left + 2 * (x >> 1);
        U = surf(1, 1, (top >> 1) + (y >> 1), b);
        V = surf(1, 1, (top >> 1) + (y >> 1), b + 1);
        break;
      }
      default:
        out[0] = out[1] = out[2] = Y;
        return;
    }
    csc_pixel(Y, U, V, out);
  }
};

__global__ __launch_bounds__(256) void k_output(const RjImageDev *__restrict__ imgs, const RjJobDev *__restrict__ jobs,
                                                int njobs, const uint8_t *__restrict__ planes) {
  const uint32_t row_g = blockIdx.x;
  const int j = upper_index(njobs, row_g, [&](int k) { return jobs[k].row_prefix; });
  const RjJobDev jb = jobs[j];
  const uint32_t row = row_g - jb.row_prefix;
  PlaneView pv{planes, &imgs[jb.image]};
  uint8_t *dst = jb.dst + uint64_t(row) * jb.dst_pitch;
  const int64_t sr = int64_t(jb.src_row0) + row;
  const int sp = jb.chan_sel & 15, chan = (jb.chan_sel >> 4) & 15, stride = jb.chan_sel >> 8;
  for (uint32_t x = threadIdx.x; x < jb.row_bytes; x += 256) {
    uint8_t v;
    switch (jb.kind) {
      case RJ_JOB_COPY:
        v = pv.surf(sp, chan, sr, int64_t(jb.src_byte0) + x);
        break;
      case RJ_JOB_CHROMA:
        v = pv.surf(sp, chan, sr, int64_t(jb.src_byte0) + int64_t(stride) * x);
        break;
      case RJ_JOB_Y:
        v = pv.px(0, sr, int64_t(jb.src_byte0) + x);
        break;
      case RJ_JOB_RGB: {
        uint8_t p[3];
        pv.rgb(row, x / 3, p);
        v = p[x % 3];
        break;
      }
      default: {  // RJ_JOB_RGB_PLANE
        uint8_t p[3];
        pv.rgb(row, x, p);
        v = p[chan];
        break;
      }
    }
    gp(dst)[x] = v;
  }
}

hipError_t LaunchOutputJobs(hipStream_t st, const RjImageDev *imgs, const RjJobDev *jobs, int njobs, uint32_t total_rows,
                            const uint8_t *planes) {
  if (total_rows == 0 || njobs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_output, dim3(total_rows), dim3(256), 0, st, imgs, jobs, njobs, planes);
  return hipGetLastError();
}

}  // namespace rj
