// rj_kernels.hip -- the JPEG decode hot path for MI355X (gfx950, wave64).
//
// Replaces the VCN fixed-function decode of the reference (src/rocjpeg_vaapi_decoder.cpp:
// 574-692) and rewrites its post-processing kernels (src/rocjpeg_hip_kernels.cpp).
//
//   K0 k_destuff      one wavefront per restart interval: coalesced byte loads, FF00/fill
//                     removal by per-lane keep masks + wave prefix sum, compacted stores.
//   K1 k_huffman      one lane per restart interval: LDS bit ring + two-level LDS LUT,
//                     flattened symbol loop (lanes never wait for each other at block
//                     boundaries), sparse entry stream staged in LDS, 64-B group stores.
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
// index of the last entry with prefix <= key (prefix[0] == 0, monotone)
template <typename F>
__device__ __forceinline__ int upper_index(int n, uint32_t key, F prefix_of) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (prefix_of(mid) <= key) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ uint32_t wave_exclusive_scan(uint32_t v, uint32_t lane, uint32_t &total) {
  uint32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    if (lane >= uint32_t(off)) x += y;
  }
  total = __shfl(x, 63, 64);
  return x - v;
}

// ---------------------------------------------------------------------------------------
// K0: destuff.  Within an interval's raw range the host guarantees only data bytes,
// FF 00 pairs and FF fill runs in front of an FF 00 occur.  Byte i is dropped when
// (b[i] == 00 && b[i-1] == FF) or (b[i] == FF && b[i+1] == FF).
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_destuff(const RjImageDev *__restrict__ imgs, int nimg,
                                                uint8_t *__restrict__ destuffed, uint32_t *__restrict__ seg_len) {
  const uint32_t g = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const int i = upper_index(nimg, g, [&](int k) { return imgs[k].seg_prefix; });
  const RjImageDev &im = imgs[i];
  const RjSegDev sg = gp(im.segs)[g - im.seg_prefix];
  const RJ_GLOBAL uint8_t *src = gp(im.ecs + sg.src_off);
  uint8_t *dst = destuffed + im.destuff_off + sg.dst_off;
  const uint32_t len = sg.src_len;
  uint32_t out = 0;
  uint32_t prev_byte = 0;  // byte before the current 256-B chunk
  for (uint32_t base = 0; base < len; base += 256) {
    const uint32_t p = base + 4 * lane;
    uint32_t b[4];
#pragma unroll
    for (int k = 0; k < 4; k++) b[k] = (p + k < len) ? src[p + k] : 0x100u;  // 0x100 = past the end
    const uint32_t nb_next = (base + 256 < len) ? src[base + 256] : 0x100u;
    uint32_t prev = __shfl_up(b[3], 1, 64);
    if (lane == 0) prev = prev_byte;
    uint32_t next = __shfl_down(b[0], 1, 64);
    if (lane == 63) next = nb_next;
    uint32_t keep = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t pv = k == 0 ? prev : b[k - 1];
      const uint32_t nx = k == 3 ? next : b[k + 1];
      const bool drop = b[k] == 0x100u || (b[k] == 0x00u && pv == 0xFFu) || (b[k] == 0xFFu && nx == 0xFFu);
      keep |= (drop ? 0u : 1u) << k;
    }
    uint32_t total;
    uint32_t o = wave_exclusive_scan(__popc(keep), lane, total) + out;
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (keep & (1u << k)) dst[o++] = uint8_t(b[k]);
    out += total;
    prev_byte = __shfl(b[3], 63, 64);
  }
  // zero the slack after the data (>= 16 B, see rj_stream.cpp BuildPlan): K1 reads whole 16-B
  // chunks and must see zero bits past the end, as libjpeg inserts after a marker
  const uint32_t pad_end = (len + 16u + 15u) & ~15u;
  for (uint32_t b = out + lane; b < pad_end; b += 64) dst[b] = 0;
  if (lane == 0) seg_len[g] = out;
}

hipError_t LaunchDestuff(hipStream_t st, const RjImageDev *imgs, int nimg, uint32_t nseg, uint8_t *destuffed,
                         uint32_t *seg_len) {
  if (nseg == 0) return hipSuccess;
  hipLaunchKernelGGL(k_destuff, dim3(nseg), dim3(64), 0, st, imgs, nimg, destuffed, seg_len);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// K1: Huffman decode, one lane per restart interval (T.81 F.2.2, libjpeg jdhuff.c semantics).
//
// Per lane everything on the per-symbol dependency chain stays on-chip:
//   * bits: a 64-bit MSB-first buffer refilled 32 bits at a time from a per-lane LDS ring of
//     the interval's destuffed bytes; the next ring word is read one symbol ahead, so the only
//     LDS round trip left on the chain is the Huffman lookup itself.  The ring is topped up
//     from HBM at wave-uniform phase boundaries (every RJ_PHASE symbols) with loads issued one
//     phase before they are committed, so their latency hides behind a whole phase of decoding
//     (a conditional global load inside the loop would cost a full vmcnt(0) round trip).
//   * lookup: two-level LUT in LDS (9-bit first level + 7-bit second level, rj_device.h); the
//     extra bits come from the same 32-bit peek (v_bfe_u32), HUFF_EXTEND branch-free.
//   * output: entries are staged in a per-lane LDS ring and leave in 64-B groups at phase
//     boundaries (4 x 16-B stores) -- no per-symbol global store, no per-block index.
// The flattened symbol loop lets every lane run at its own pace across block boundaries.
// ---------------------------------------------------------------------------------------
#define RJ_RING_CHUNKS 12  // 16-B chunks per lane in the bit ring (192 B)
#define RJ_RING_WORDS (RJ_RING_CHUNKS * 4)
#define RJ_PHASE 16         // symbols per phase: <= 16 ring words consumed (<= 32 bits/symbol)
#define RJ_PREFETCH 4       // chunks fetched per phase at most
#define RJ_STAGE 32         // staged entries per lane (two 64-B groups)
// Ring invariant: after every phase commit the ring holds >= 17 unread words (or all that is
// left).  With U unread words, a phase prefetches n = min(4, 12 - used) chunks and consumes at
// most 16 words, so U' = U - 16 + 4n >= min(U, 28) -- the symbol loop never reads HBM.

struct BitReader {
  const uint4 *src;   // 16-B aligned destuffed bytes, zero-padded after nbytes
  uint32_t *ring;     // this lane's LDS ring (RJ_RING_WORDS words)
  uint32_t nchunks;   // 16-B chunks holding data
  uint32_t rd;        // words moved into the bit buffer (monotonic)
  uint32_t rdw;       // rd mod RJ_RING_WORDS
  uint32_t cm;        // chunks committed to the ring (monotonic)
  uint32_t cms;       // cm mod RJ_RING_CHUNKS
  uint32_t pn;        // chunks in the pending prefetch
  uint4 pf[RJ_PREFETCH];
  uint32_t nw;        // ring word rd, read ahead
  int nb;             // valid bits in acc (left-justified)
  uint64_t acc;

  __device__ __forceinline__ void init(const uint4 *s, uint32_t *r, uint32_t nbytes) {
    src = s;
    ring = r;
    nchunks = (nbytes + 15) / 16;
    const uint32_t first = nchunks < RJ_RING_CHUNKS ? nchunks : RJ_RING_CHUNKS;
    for (uint32_t q = 0; q < first; q++) reinterpret_cast<uint4 *>(ring)[q] = src[q];
    cm = first;
    cms = first == RJ_RING_CHUNKS ? 0 : first;
    rd = 0;
    rdw = 0;
    pn = 0;
#pragma unroll
    for (int q = 0; q < RJ_PREFETCH; q++) pf[q] = make_uint4(0, 0, 0, 0);
    nw = ring[0];
    nb = 0;
    acc = 0;
  }
  // phase boundary: commit the previous prefetch (loaded one phase ago), issue the next one
  // (loads unconditional, clamped: a conditional load would force an immediate wait)
  __device__ __forceinline__ void phase() {
#pragma unroll
    for (int q = 0; q < RJ_PREFETCH; q++)
      if (uint32_t(q) < pn) {
        reinterpret_cast<uint4 *>(ring)[cms] = pf[q];
        cms = cms == RJ_RING_CHUNKS - 1 ? 0 : cms + 1;
      }
    cm += pn;
    const uint32_t used = cm - (rd >> 2);  // live chunks, incl. the one being read
    const uint32_t room = RJ_RING_CHUNKS - used;
    uint32_t want = nchunks > cm ? nchunks - cm : 0u;
    want = want < room ? want : room;
    pn = want < RJ_PREFETCH ? want : RJ_PREFETCH;
    const uint32_t last = nchunks ? nchunks - 1 : 0;
#pragma unroll
    for (int q = 0; q < RJ_PREFETCH; q++) pf[q] = src[cm + q < last ? cm + q : last];
    nw = ring[rdw];  // the commit may have landed the read-ahead word
  }
  __device__ __forceinline__ void refill() {
    if (nb <= 32) {
      const uint32_t w = rd < 4 * cm ? nw : 0u;  // past the data: zero bits, as libjpeg inserts
      acc |= uint64_t(__builtin_bswap32(w)) << (32 - nb);
      nb += 32;
      rd++;
      rdw = rdw == RJ_RING_WORDS - 1 ? 0 : rdw + 1;
    }
    nw = ring[rdw];
  }
  __device__ __forceinline__ bool overrun(uint32_t nbytes) const {
    return uint64_t(rd) * 32u - uint64_t(nb) > uint64_t(nbytes) * 8u;
  }
};

// canonical search for codes the LDS tables do not resolve (second-level pool exhausted, or a
// DC code longer than 9 bits): libjpeg jpeg_huff_decode on the table in HBM
__device__ __forceinline__ uint32_t huff_slow(const RjHuffDev *t, uint32_t peek16) {
  uint32_t e = RJ_LUT_BAD;
  for (int l = 1; l <= 16; l++)
    if (peek16 < t->maxcode16[l]) {
      e = uint32_t(l << 8) | t->vals[((peek16 >> (16 - l)) + t->valoff[l]) & 255];
      break;
    }
  return e;
}

// LDS table image: DC tables first level only (512 entries each), AC tables both levels
#define RJ_SLUT_AC0 (2 * RJ_LUT_L1)
#define RJ_SLUT_ENTRIES (2 * RJ_LUT_L1 + 2 * RJ_LUT_ENTRIES)

__global__ __launch_bounds__(64) void k_huffman(const RjImageDev *__restrict__ imgs, int nimg, uint32_t nseg,
                                                const uint8_t *__restrict__ destuffed,
                                                const uint32_t *__restrict__ seg_len,
                                                const RjTableSet *__restrict__ tabsets, RjCoefBuf coefs) {
  // strides padded by 16 B so the 8-lane groups of ds_*_b128 hit distinct banks
  __shared__ __attribute__((aligned(16))) uint32_t s_ring[64][RJ_RING_WORDS + 4];
  __shared__ __attribute__((aligned(16))) uint32_t s_stage[64][RJ_STAGE + 4];
  __shared__ __attribute__((aligned(16))) uint16_t s_lut[RJ_SLUT_ENTRIES];
  const uint32_t lane = threadIdx.x;
  const uint32_t g = blockIdx.x * 64u + lane;
  const bool valid = g < nseg;
  const int i = valid ? upper_index(nimg, g, [&](int k) { return imgs[k].seg_prefix; }) : 0;
  const RjImageDev &im = imgs[i];
  const uint32_t my_ts = im.tabset;
  bool pending = valid;
  // one pass per distinct table set among the wave's lanes (normally exactly one)
  while (true) {
    const uint64_t m = __ballot(pending);
    if (m == 0) break;
    const uint32_t T = __shfl(my_ts, __ffsll((long long)m) - 1, 64);
    __syncthreads();
    {
      const RjTableSet &ts = tabsets[T];
      uint4 *d4 = reinterpret_cast<uint4 *>(s_lut);
      constexpr uint32_t L1Q = RJ_LUT_L1 * 2 / 16, FQ = RJ_LUT_ENTRIES * 2 / 16;
      for (uint32_t k = lane; k < 2 * L1Q + 2 * FQ; k += 64) {
        const uint4 *s4;
        if (k < L1Q) s4 = reinterpret_cast<const uint4 *>(ts.dc[0].lut) + k;
        else if (k < 2 * L1Q) s4 = reinterpret_cast<const uint4 *>(ts.dc[1].lut) + (k - L1Q);
        else if (k < 2 * L1Q + FQ) s4 = reinterpret_cast<const uint4 *>(ts.ac[0].lut) + (k - 2 * L1Q);
        else s4 = reinterpret_cast<const uint4 *>(ts.ac[1].lut) + (k - 2 * L1Q - FQ);
        d4[k] = *s4;
      }
    }
    __syncthreads();
    if (pending && my_ts == T) {
      pending = false;
      const RjSegDev sg = gp(im.segs)[g - im.seg_prefix];
      const uint32_t nblk = im.nblk_mcu, mcux = im.mcux;
      // per block-in-MCU b: component (2 bits) | dc table (1) | ac table (1), 4 bits each
      uint64_t binfo = 0;
      for (uint32_t b = 0; b < nblk; b++) {
        const uint32_t c = im.blk_comp[b] & 3;
        binfo |= uint64_t(c | ((im.comp_td[c] & 1) << 2) | ((im.comp_ta[c] & 1) << 3)) << (4 * b);
      }
      const uint32_t nbytes = seg_len[g];
      BitReader br;
      br.init(reinterpret_cast<const uint4 *>(destuffed + im.destuff_off + sg.dst_off), s_ring[lane], nbytes);
      uint32_t *const ent = coefs.ent + im.ent_off + sg.ent_off;  // group-aligned region
      uint32_t *const stage = s_stage[lane];
      uint32_t ne = 0, fl = 0;  // entries produced / flushed (fl multiple of RJ_ENT_GROUP)

      // MCU row checkpoints for K2
      const uint32_t row0 = im.row_off;
      uint32_t mrow = sg.mcu_first / mcux;
      uint32_t to_row = mcux - (sg.mcu_first - mrow * mcux);  // MCUs until the next row starts
      if (to_row == mcux) gp(coefs.row)[row0 + mrow] = sg.ent_off;

      int pred0 = 0, pred1 = 0, pred2 = 0;
      bool skip = (sg.flags & RJ_SEG_MISSING) != 0;
      uint32_t blocks_left = sg.mcu_count * nblk;
      uint32_t b = 0;
      uint32_t info = uint32_t(binfo) & 15u;
      int k = 0;
      uint32_t dcbase = ((info >> 2) & 1u) * RJ_LUT_L1, acbase = RJ_SLUT_AC0 + ((info >> 3) & 1u) * RJ_LUT_ENTRIES;
      uint32_t iter = 0;
      while (blocks_left > 0) {
        if ((iter++ & (RJ_PHASE - 1)) == 0) {  // phase boundary: same count in every active lane
          br.phase();
          if (ne - fl >= RJ_ENT_GROUP) {  // one full 64-B group leaves the stage
            const uint4 *s4 = reinterpret_cast<const uint4 *>(stage + (fl & (RJ_STAGE - 1)));
            uint4 *d4 = reinterpret_cast<uint4 *>(ent + fl);
#pragma unroll
            for (int q = 0; q < RJ_ENT_GROUP / 4; q++) gp(d4)[q] = s4[q];
            fl += RJ_ENT_GROUP;
          }
        }
        {
          uint32_t entry;
          bool emit;
          if (skip) {  // libjpeg: the rest of the interval decodes to zero blocks
            entry = 0;
            emit = true;
            k = 64;
          } else {
            br.refill();
            const uint32_t c = info & 3u;
            const uint32_t peek32 = uint32_t(br.acc >> 32);
            // LDS table base: DC tables (first level only) at 0 / 512, AC tables after them
            const uint32_t tbase = k == 0 ? dcbase : acbase;
            uint32_t e = s_lut[tbase + (peek32 >> 23)];
            if (e & 0x8000u) {
              if (e != 0xFFFFu && k != 0) {
                e = s_lut[tbase + RJ_LUT_L1 + (e & 0x7Fu) * 128u + ((peek32 >> 16) & 127u)];
              } else {
                const RjHuffDev *t = k == 0 ? &tabsets[T].dc[(info >> 2) & 1u] : &tabsets[T].ac[(info >> 3) & 1u];
                e = huff_slow(t, peek32 >> 16);
              }
            }
            const uint32_t len = e >> 8, sym = e & 255u;
            const uint32_t s = sym & 15u, r = sym >> 4;
            // extra bits follow the code inside the same peek (len + s <= 31); width 0 -> 0
            const uint32_t raw = __builtin_amdgcn_ubfe(peek32, 32u - len - s, s);
            // HUFF_EXTEND (jdhuff.h): negative when the top extra bit is 0; s == 0 gives 0
            const int val = int(raw) + (int32_t(raw - (1u << ((s - 1) & 31))) >> 31 & int32_t(1u - (1u << s)));
            br.acc <<= (len + s);
            br.nb -= int(len + s);
            // DC (k == 0): predictor per component (F.2.1.3); AC: run/size (F.2.2.2)
            const bool isdc = k == 0;
            const int p = (c == 0 ? pred0 : (c == 1 ? pred1 : pred2)) + val;
            pred0 = (isdc && c == 0) ? p : pred0;
            pred1 = (isdc && c == 1) ? p : pred1;
            pred2 = (isdc && c == 2) ? p : pred2;
            const int kk = isdc ? 0 : k + int(r);  // zigzag position of this coefficient
            entry = (uint32_t(isdc ? p : val) & 0xFFFFu) | (uint32_t(kk < 63 ? kk : 63) << 16);
            emit = isdc || s;
            k = isdc ? 1 : (s ? kk + 1 : (r == 15 ? k + 16 : 64));  // ZRL / EOB
          }
          stage[ne & (RJ_STAGE - 1)] = entry;  // a non-emitted write lands in the next free slot
          ne += emit ? 1u : 0u;
          if (k >= 64) {  // block complete
            k = 0;
            blocks_left--;
            if (++b == nblk) {
              b = 0;
              if (!skip && br.overrun(nbytes)) skip = true;  // libjpeg: rest of the interval stays zero
              if (--to_row == 0) {  // the next MCU starts a row
                to_row = mcux;
                mrow++;
                if (blocks_left) gp(coefs.row)[row0 + mrow] = sg.ent_off + ne;
              }
            }
            info = uint32_t(binfo >> (4 * b)) & 15u;
            dcbase = ((info >> 2) & 1u) * RJ_LUT_L1;
            acbase = RJ_SLUT_AC0 + ((info >> 3) & 1u) * RJ_LUT_ENTRIES;
          }
        }
      }
      // terminator, then everything still staged (whole groups; the slack is reserved)
      stage[ne & (RJ_STAGE - 1)] = RJ_ENT_TERM;
      ne++;
      while (fl < ne) {
        const uint4 *s4 = reinterpret_cast<const uint4 *>(stage + (fl & (RJ_STAGE - 1)));
        uint4 *d4 = reinterpret_cast<uint4 *>(ent + fl);
#pragma unroll
        for (int q = 0; q < RJ_ENT_GROUP / 4; q++) gp(d4)[q] = s4[q];
        fl += RJ_ENT_GROUP;
      }
    }
  }
}

hipError_t LaunchHuffman(hipStream_t st, const RjImageDev *imgs, int nimg, uint32_t nseg, const uint8_t *destuffed,
                         const uint32_t *seg_len, const RjTableSet *tabsets, RjCoefBuf coefs) {
  if (nseg == 0) return hipSuccess;
  hipLaunchKernelGGL(k_huffman, dim3((nseg + 63) / 64), dim3(64), 0, st, imgs, nimg, nseg, destuffed, seg_len, tabsets,
                     coefs);
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
