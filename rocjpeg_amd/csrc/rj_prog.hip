// rj_prog.hip -- K1p: progressive (SOF2) Huffman decode into dense coefficients.
//
// Beyond the reference (its parser rejects SOF2, src/rocjpeg_parser.cpp:74-104); SURVEY.md 8f
// rank 2 / BASELINE config C5.  Semantics restate libjpeg 9.4 jdhuff.c decode_mcu_DC_first,
// decode_mcu_AC_first, decode_mcu_DC_refine, decode_mcu_AC_refine and process_restart, as the
// CPU oracle does (oracle/jpeg_oracle.c prog_block / decode_progressive, pinned against
// libjpeg's jpeg_read_coefficients):
//   * a needed bit past the interval's data reads as 0; after the unit (MCU) in which that
//     happened the rest of the interval is skipped (coefficients keep their values);
//   * an interval whose RST marker is missing is skipped;
//   * EOB runs (AC first: 2^r + bits - 1 further blocks; AC refine: 2^r + bits blocks incl.
//     the current one), correction bits for every already-nonzero coefficient passed.
//
// Work unit: one lane per restart interval of one scan (rj_stream plan RjProgIvalDev).  The
// host launches one grid per dependency level (scans of a level touch disjoint (component,
// coefficient) pairs) and groups the lanes of a wave by scan kind, so the kind is
// wave-uniform.  Coefficients (rj_device.h): 32 dwords per block, zigzag order, DC two's
// complement, AC sign-magnitude; first scans store halfwords, refinements OR bits in (global
// atomics: two lanes of one level may share a dword across band edges).
//
// Per lane everything on the symbol chain is on-chip: the first-level LUT of the lane's table
// (9 bits; DC first: two 8-bit tables) in a lane-interleaved LDS column and the bitstream in a
// 32-word LDS ring, topped up at wave-uniform phase boundaries with loads issued one phase before
// they are committed; the symbol loop itself reads no HBM.  AC refinements are decoded by
// k_prog_wave below (a lane-per-interval refinement decoder, round 1's lane_ac_refine, measured
// 2x slower than the wave decoder in round 4 and was removed).
#include <hip/hip_runtime.h>

#include "rj_device.h"
#include "rj_kernels.h"
#include "rj_math.h"

namespace rj {

#define RJ_PW 64       // one wave per workgroup
#define RJ_PPHASE 8    // iterations per phase; an iteration consumes <= 32 bits and <= 1 block
#define RJ_PRING 32    // bit ring words per lane
#define RJ_PVALS 48    // symbol words per lane (AC tables: <= 162 symbols)

struct PRow {  // lane-interleaved LDS column: word w of this lane at base[w * 64]
  uint32_t *base;
  __device__ __forceinline__ uint32_t &operator[](uint32_t w) const { return base[w * RJ_PW]; }
};
struct HRow {
  uint16_t *base;
  __device__ __forceinline__ uint16_t &operator[](uint32_t e) const { return base[e * RJ_PW]; }
};

// MSB-first bits of one interval's destuffed data; zero past the data (as libjpeg inserts).
struct PBits {
  const uint4 *src;  // 16-B aligned interval start
  PRow ring;
  uint32_t nwords;   // words holding data
  uint32_t lastc;    // last loadable 16-B chunk
  uint32_t top;      // words committed (multiple of 4)
  uint32_t pos;      // bits consumed
  __device__ __forceinline__ void put(const uint4 &v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; q++) {
      ring[(top + q) & (RJ_PRING - 1)] = (top + q) < nwords ? __builtin_bswap32(w[q]) : 0u;
    }
    top += 4;
  }
  __device__ __forceinline__ void init(const uint4 *s, PRow r, uint32_t len) {
    src = s;
    ring = r;
    nwords = (len + 3) / 4;
    lastc = len ? (len - 1) / 16 : 0u;
    top = 0;
    pos = 0;
    uint4 v[6];
#pragma unroll
    for (uint32_t q = 0; q < 6; q++) v[q] = gp(src)[min(q, lastc)];
#pragma unroll
    for (int q = 0; q < 6; q++) put(v[q]);
  }
  __device__ __forceinline__ uint32_t peek() const {
    const uint32_t w = pos >> 5;
    const uint64_t x = (uint64_t(ring[w & (RJ_PRING - 1)]) << 32) | ring[(w + 1) & (RJ_PRING - 1)];
    return uint32_t((x << (pos & 31)) >> 32);
  }
  // a phase consumes <= 8 words; the ring keeps >= 9 unread words at every phase start
  __device__ __forceinline__ bool room() const { return top + 8 - (pos >> 5) <= RJ_PRING; }
  __device__ __forceinline__ void issue(uint4 &a, uint4 &b) const {
    a = gp(src)[min(top / 4, lastc)];
    b = gp(src)[min(top / 4 + 1, lastc)];
  }
  __device__ __forceinline__ void commit(const uint4 &a, const uint4 &b, bool n) {
    if (n) {
      put(a);
      put(b);
    }
  }
};

// global-address-space stores / atomics (generic FLAT ones would count in lgkmcnt and stall
// every LDS wait of the symbol loop, rj_math.h gp)
__device__ __forceinline__ void gst16(uint16_t *p, uint32_t v) { *gp(p) = uint16_t(v); }
__device__ __forceinline__ void gor32(uint32_t *p, uint32_t v) {
  __hip_atomic_fetch_or(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gor64(unsigned long long *p, unsigned long long v) {
  __hip_atomic_fetch_or(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t pbits(uint32_t peek, uint32_t off, uint32_t n) {  // off + n <= 32
  return n ? (peek << off) >> (32u - n) : 0u;
}
__device__ __forceinline__ int32_t pextend(uint32_t v, uint32_t s) {
  return (s && v < (1u << (s - 1))) ? int32_t(v) - int32_t(1u << s) + 1 : int32_t(v);
}

// Codes longer than the LDS first level: canonical decode from per-lane registers (libjpeg
// jpeg_huff_decode restated).  Left-justified to 16 bits, the codes of length l fill
// [mc(l-1), mc(l)), mc = the monotone exclusive bound of all codes of length <= l; no global
// access on the symbol chain (a wave in which any lane met a long code would otherwise wait a
// full memory latency -- and with 64 lanes that is nearly every iteration).  The symbols sit in
// the lane's LDS column (VRow); a code past mc(16) is libjpeg's bad code (17 bits, symbol 0).
struct VRow {
  uint32_t *base;
  __device__ __forceinline__ uint32_t &operator[](uint32_t w) const { return base[w * RJ_PW]; }
  __device__ __forceinline__ uint32_t byte(uint32_t b) const { return ((*this)[b >> 2] >> ((b & 3u) * 8u)) & 255u; }
};
struct PLong {
  uint32_t mc[8];  // bound for lengths 9..16
  int32_t vo[8];   // symbol index = code + vo[l - 9]
  uint32_t vbase;  // this table's first symbol byte in the lane's VRow
  __device__ __forceinline__ void load(const RjHuffDev *t, uint32_t vb) {
    uint32_t m = 0;
#pragma unroll
    for (int l = 1; l <= 16; l++) {
      m = max(m, gp(t->maxcode16)[l]);
      if (l >= 9) mc[l - 9] = m;
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
      vo[j] = gp(t->valoff)[9 + j];
    }
    vbase = vb;
  }
};
__device__ __forceinline__ uint32_t plong_decode(const PLong &a, uint32_t peek, const VRow &vals) {
  const uint32_t p16 = peek >> 16;
  // the bounds are monotone, so with ge_j = (p16 >= mc[j]): l = 9 + sum ge_j and
  // vo[l - 9] = vo[0] + sum ge_j * (vo[j+1] - vo[j]) -- masks, no select of loads (which the
  // backend turns into a scratch array)
  uint32_t l = 9;
  int32_t vo = a.vo[0];
#pragma unroll
  for (int j = 0; j < 7; j++) {
    const uint32_t m = 0u - (p16 >= a.mc[j] ? 1u : 0u);
    l += m & 1u;
    vo += int32_t(uint32_t(a.vo[j + 1] - a.vo[j]) & m);
  }
  const uint32_t idx = uint32_t(int32_t(p16 >> (16u - l)) + vo) & 255u;
  const uint32_t sym = vals.byte(a.vbase + idx);
  return p16 >= a.mc[7] ? RJ_LUT_BAD : ((l << 8) | sym);
}
// symbols of a table into the lane's VRow words [w0, w0 + nw)
__device__ __forceinline__ void load_vals(const RjHuffDev *t, const VRow &vals, uint32_t w0, uint32_t nw) {
  const uint32_t *src = reinterpret_cast<const uint32_t *>(t->vals);
  for (uint32_t w = 0; w < nw; w++) vals[w0 + w] = gp(src)[w];
}

// ---- lane geometry shared by the kinds ----
struct PGeo {
  uint32_t coef;          // block raster: dword index of block (0,0) of each scan component = cbase
  uint32_t cb[3], wb[3];  // per scan component: dense block base, raster width
  uint32_t hs[3], vs[3];
  uint32_t ns, units_x;
  uint32_t ux, uy, u, nunits;
};

__device__ __forceinline__ uint32_t sel3(uint32_t i, uint32_t a, uint32_t b, uint32_t c) { return i == 0 ? a : (i == 1 ? b : c); }

// block index (dense raster of the image) of slot (ci, dx, dy) of unit (ux, uy)
__device__ __forceinline__ uint32_t pblock(const PGeo &g, uint32_t ci, uint32_t dx, uint32_t dy) {
  const uint32_t h = sel3(ci, g.hs[0], g.hs[1], g.hs[2]), v = sel3(ci, g.vs[0], g.vs[1], g.vs[2]);
  const uint32_t b = sel3(ci, g.cb[0], g.cb[1], g.cb[2]), w = sel3(ci, g.wb[0], g.wb[1], g.wb[2]);
  return b + (g.uy * v + dy) * w + g.ux * h + dx;
}
__device__ __forceinline__ void unit_step(PGeo &g, uint32_t n) {
  g.u += n;
  g.ux += n;
  if (g.ux >= g.units_x) {
    g.uy += g.ux / g.units_x;
    g.ux = g.ux % g.units_x;
  }
}

struct PLaneIn {
  const RjImageDev *im;
  RjProgScanDev sc;
  RjProgIvalDev iv;
  bool active;
};

// ---------------------------------------------------------------------------------------
// DC first / DC refine (possibly interleaved): one block per iteration
// ---------------------------------------------------------------------------------------
template <bool kRefine>
__device__ __forceinline__ void lane_dc(const PLaneIn &L, PGeo &g, PBits &br, const HRow &lut, const VRow &vals, uint16_t *coef16,
                        unsigned long long *rec) {
  const RjProgScanDev &sc = L.sc;
  if constexpr (kRefine) {
    // DC refinement has no Huffman codes: block i of the interval (decode order) takes stream bit
    // i, and libjpeg reads zeros past the data.  The record words are therefore the stream's bits
    // in order -- word w = bit-reversed big-endian bytes [8w, 8w + 8) -- cut at min(data bits,
    // blocks): a copy, not a walk (the block-by-block loop below took ~30 ms per 1080p image).
    if (!L.active) return;
    uint32_t per = 0;
    for (uint32_t q = 0; q < g.ns && q < 3; q++) per += g.hs[q] * g.vs[q];
    const uint32_t lim = min(g.nunits * per, L.iv.dst_len * 8u);
    const uint2 *src = reinterpret_cast<const uint2 *>(br.src);  // the interval start is 16-B aligned
    for (uint32_t w = 0; w * 64u < lim; w++) {
      const uint2 v = gp(src)[w];  // the destuffed interval has >= 16 zero bytes of slack after its data
      const uint64_t x = (uint64_t(__builtin_bswap32(v.x)) << 32) | __builtin_bswap32(v.y);
      uint64_t bits = __builtin_bitreverse64(x);
      const uint32_t left = lim - w * 64u;
      if (left < 64u) bits &= (1ull << left) - 1ull;
      *gp(rec + w) = bits;
    }
    return;
  }
  const RjHuffDev *gt0 = nullptr, *gt1 = nullptr;
  if (!kRefine && L.active) {
    gt0 = L.im->ptabs + sc.tab[0];
    gt1 = L.im->ptabs + (sc.tab[1] == 0xFFFFu ? sc.tab[0] : sc.tab[1]);
    // 8-bit first levels of both tables: entry = the 9-bit entry when the code has <= 8 bits
    for (uint32_t t = 0; t < 2; t++) {
      const uint4 *src = reinterpret_cast<const uint4 *>((t ? gt1 : gt0)->lut);
      for (uint32_t q = 0; q < 64; q++) {
        const uint4 v = gp(src)[q];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t e = w[j] & 0xFFFFu;  // even entry of the pair: index 2p
          lut[t * 256u + q * 4u + j] = uint16_t(((e & 0x8000u) == 0 && (e >> 8) <= 8u) ? e : 0x8000u);
        }
      }
    }
  }
  PLong lg0, lg1;  // DC codes longer than 8 bits (12 symbols per table: 16-byte slots)
  if (!kRefine && L.active) {
    lg0.load(gt0, 0);
    lg1.load(gt1, 16);
    load_vals(gt0, vals, 0, 4);
    load_vals(gt1, vals, 4, 4);
  }
  const uint32_t al = sc.al;
  const uint32_t tsel = uint32_t(sc.tsel[0]) | (uint32_t(sc.tsel[1]) << 1) | (uint32_t(sc.tsel[2]) << 2);
  const uint32_t nbits = L.iv.dst_len * 8u;
  int32_t pred0 = 0, pred1 = 0, pred2 = 0;
  uint32_t ci = 0, dx = 0, dy = 0;
  uint64_t bacc = 0;   // DC refinement: one bit per block of the interval, in decode order
  uint32_t bn = 0, bw = 0;
  bool active = L.active;
  while (__any(active)) {
    uint4 pa, pb;
    const bool rb = br.room();
    br.issue(pa, pb);
#pragma unroll 1
    for (int it = 0; it < RJ_PPHASE; it++) {
      if (!active) continue;
      const uint32_t peek = br.peek();
      const uint32_t blk = pblock(g, ci, dx, dy);
      if (kRefine) {
        (void)blk;
        bacc |= uint64_t(peek >> 31) << bn;
        br.pos += 1;
        if (++bn == 64) {
          *gp(rec + bw) = bacc;
          bw++;
          bn = 0;
          bacc = 0;
        }
      } else {
        const uint32_t t = (tsel >> ci) & 1u;
        uint32_t e = lut[(t << 8) | (peek >> 24)];
        if (e & 0x8000u) {  // element-wise select (a reference select would put both in scratch)
          PLong a;
#pragma unroll
          for (int j = 0; j < 8; j++) {
            a.mc[j] = t ? lg1.mc[j] : lg0.mc[j];
            a.vo[j] = t ? lg1.vo[j] : lg0.vo[j];
          }
          a.vbase = t ? 16u : 0u;
          e = plong_decode(a, peek, vals);
        }
        const uint32_t len = e >> 8, s = e & 15u;
        const int32_t diff = pextend(pbits(peek, len, s), s);
        int32_t p;
        if (ci == 0) p = pred0 += diff;
        else if (ci == 1) p = pred1 += diff;
        else p = pred2 += diff;
        gst16(coef16 + (g.coef + blk * 32u) * 2u, uint32_t(p) << al);
        br.pos += len + s;
      }
      // next slot of the unit
      const uint32_t h = sel3(ci, g.hs[0], g.hs[1], g.hs[2]), v = sel3(ci, g.vs[0], g.vs[1], g.vs[2]);
      if (++dx == h) {
        dx = 0;
        if (++dy == v) {
          dy = 0;
          if (++ci == g.ns) {
            ci = 0;
            unit_step(g, 1);
            if (g.u >= g.nunits || br.pos > nbits) {
              active = false;
              if (kRefine && bn) *gp(rec + bw) = bacc;  // the interval's last, partial word
            }
          }
        }
      }
    }
    br.commit(pa, pb, rb);
  }
}

// ---------------------------------------------------------------------------------------
// AC first (one component): one symbol (or one EOB-run skip) per iteration
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void lane_ac_first(const PLaneIn &L, PGeo &g, PBits &br, const HRow &lut, const VRow &vals,
                              uint16_t *coef16, unsigned long long *nz, uint32_t nzbase) {
  const RjProgScanDev &sc = L.sc;
  const RjHuffDev *gt = L.active ? L.im->ptabs + sc.tab[0] : nullptr;
  if (L.active) {
    const uint4 *src = reinterpret_cast<const uint4 *>(gt->lut);
    for (uint32_t q = 0; q < 64; q++) {
      const uint4 v = gp(src)[q];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        lut[q * 8u + 2 * j] = uint16_t(w[j] & 0xFFFFu);
        lut[q * 8u + 2 * j + 1] = uint16_t(w[j] >> 16);
      }
    }
  }
  PLong lg;  // AC codes longer than 9 bits
  if (L.active) {
    lg.load(gt, 0);
    load_vals(gt, vals, 0, RJ_PVALS);
  }
  const uint32_t ss = sc.ss, se = sc.se, al = sc.al;
  const uint32_t nbits = L.iv.dst_len * 8u;
  uint32_t k = ss, eobrun = 0;
  uint64_t blk_nz = 0;
  bool active = L.active;
  while (__any(active)) {
    uint4 pa, pb;
    const bool rb = br.room();
    br.issue(pa, pb);
#pragma unroll 1
    for (int it = 0; it < RJ_PPHASE; it++) {
      if (!active) continue;
      if (eobrun) {  // blocks inside an EOB run: nothing coded, nothing to write
        const uint32_t n = min(eobrun, g.nunits - g.u);
        eobrun -= n;
        unit_step(g, n);
        if (g.u >= g.nunits) active = false;
        continue;
      }
      const uint32_t peek = br.peek();
      uint32_t e = lut[peek >> 23];
      const uint32_t el = plong_decode(lg, peek, vals);  // branch-free: both lookups in flight
      e = (e & 0x8000u) ? el : e;
      const uint32_t len = e >> 8, r = (e >> 4) & 15u, s = e & 15u;
      if (s) {
        // corrupt data can run past Se; such a coefficient is dropped (libjpeg would store it
        // outside the band, where another scan of this component may be writing concurrently)
        const uint32_t q = min(k + r, 63u);
        const int32_t v = pextend(pbits(peek, len, s), s);
        const uint32_t mag = (uint32_t(v < 0 ? -v : v) << al) & 0x7FFFu;
        const uint32_t blk = pblock(g, 0, 0, 0);
        if (q <= se) {
          gst16(coef16 + (g.coef + blk * 32u) * 2u + q, mag | (v < 0 ? 0x8000u : 0u));
          blk_nz |= 1ull << q;
        }
        k += r + 1;
        br.pos += len + s;
      } else if (r == 15) {
        k += 16;
        br.pos += len;
      } else {
        eobrun = r ? (1u << r) + pbits(peek, len, r) - 1u : 0u;
        k = se + 1;
        br.pos += len + r;
      }
      if (k > se) {  // block done
        if (blk_nz) gor64(nz + nzbase + g.u, blk_nz);
        blk_nz = 0;
        k = ss;
        unit_step(g, 1);
        if (g.u >= g.nunits || br.pos > nbits) active = false;
      }
    }
    br.commit(pa, pb, rb);
  }
}

// ---------------------------------------------------------------------------------------
// AC refinement (one component): one symbol and/or up to 32 bits of correction walk per
// iteration; the walk uses the block's nonzero mask (positions in [ss, se] coded earlier)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t lomask(uint32_t n) { return n >= 64 ? ~0ull : ((1ull << n) - 1); }
__device__ __forceinline__ uint32_t ctz64(uint64_t x) { return uint32_t(__builtin_ctzll(x)); }

__global__ __launch_bounds__(RJ_PW) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_prog(const RjImageDev *__restrict__ imgs, int nimg,
                                                const uint32_t *__restrict__ lanes, uint32_t nlanes,
                                                const uint8_t *__restrict__ destuffed, uint32_t *__restrict__ coef,
                                                unsigned long long *__restrict__ nz,
                                                unsigned long long *__restrict__ recs) {
  __shared__ uint16_t s_lut[RJ_LUT_L1 * RJ_PW];
  __shared__ uint32_t s_vals[RJ_PVALS * RJ_PW];
  __shared__ uint32_t s_ring[RJ_PRING * RJ_PW];
  const uint32_t lane = threadIdx.x;
  const uint32_t gl = blockIdx.x * RJ_PW + lane;
  const uint32_t gi = gl < nlanes ? *gp(lanes + gl) : 0xFFFFFFFFu;
  PLaneIn L;
  L.active = gi != 0xFFFFFFFFu;
  int i = 0;
  if (L.active) i = upper_index(nimg, gi, [&](int q) { return imgs[q].pival_prefix; });
  const RjImageDev &im = imgs[i];
  L.im = &im;
  L.sc = RjProgScanDev{};
  L.iv = RjProgIvalDev{};
  if (L.active) {
    L.iv = *gp(im.pivals + (gi - im.pival_prefix));
    L.sc = *gp(im.pscans + L.iv.scan);
    if (L.iv.flags & RJ_SEG_MISSING) L.active = false;  // libjpeg: skipped to the next marker
  }
  // the host groups lanes so that every wave holds one scan kind (lane 0 is always real)
  const uint32_t kind = __builtin_amdgcn_readfirstlane(uint32_t(L.sc.kind));

  PGeo g;
  g.coef = uint32_t(0);
  g.ns = L.sc.ns ? L.sc.ns : 1u;
  g.units_x = L.sc.units_x ? L.sc.units_x : 1u;
  g.nunits = L.active ? L.iv.nunits : 0u;
  g.u = 0;
  g.ux = L.iv.unit0 % g.units_x;
  g.uy = L.iv.unit0 / g.units_x;
#pragma unroll
  for (int q = 0; q < 3; q++) {
    const uint32_t c = L.sc.comp[q] & 3u;
    g.cb[q] = c == 0 ? im.cblk0[0] : (c == 1 ? im.cblk0[1] : im.cblk0[2]);
    g.wb[q] = c == 0 ? im.wblk[0] : (c == 1 ? im.wblk[1] : im.wblk[2]);
    g.hs[q] = L.sc.hs[q] ? L.sc.hs[q] : 1u;
    g.vs[q] = L.sc.vs[q] ? L.sc.vs[q] : 1u;
  }
  // the dense coefficients of this image: 32-bit dword offsets inside a per-image window
  uint32_t *coef32 = coef + (L.active ? im.coef_off : 0ull);
  uint16_t *coef16 = reinterpret_cast<uint16_t *>(coef32);
  const uint32_t c0 = L.sc.comp[0] & 3u;
  // nonzero masks of this interval's units: the component's raster from the interval's first unit
  const uint32_t nzbase =
      L.active ? (c0 == 0 ? im.nzblk0[0] : (c0 == 1 ? im.nzblk0[1] : im.nzblk0[2])) + L.iv.unit0 : 0u;
  unsigned long long *nzi = nz + (L.active ? im.nz_off : 0ull);
  unsigned long long *rec = recs + (L.active ? im.prec_off + L.iv.rec_off : 0ull);

  PBits br;
  const uint8_t *data = L.active ? destuffed + im.destuff_off + L.iv.dst_off : destuffed;
  br.init(reinterpret_cast<const uint4 *>(data), PRow{s_ring + lane}, L.active ? L.iv.dst_len : 0u);
  const HRow lut{s_lut + lane};
  const VRow vals{s_vals + lane};
  switch (kind) {
    case RJ_PK_DC_FIRST:
      lane_dc<false>(L, g, br, lut, vals, coef16, rec);
      break;
    case RJ_PK_DC_REFINE:
      lane_dc<true>(L, g, br, lut, vals, coef16, rec);
      break;
    case RJ_PK_AC_FIRST:
      lane_ac_first(L, g, br, lut, vals, coef16, nzi, nzbase);
      break;
    default:  // AC refinements are never given to the lanes (k_prog_wave decodes them)
      break;
  }
}

hipError_t LaunchProgressive(hipStream_t st, const RjImageDev *imgs, int nimg, const uint32_t *lanes, uint32_t nlanes,
                             const uint8_t *destuffed, uint32_t *coef, unsigned long long *nz,
                             unsigned long long *recs) {
  if (nlanes == 0) return hipSuccess;
  hipLaunchKernelGGL(k_prog, dim3((nlanes + RJ_PW - 1) / RJ_PW), dim3(RJ_PW), 0, st, imgs, nimg, lanes, nlanes,
                     destuffed, coef, nz, recs);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// k_prog_wave: AC scans, one WAVE per interval (wave-cooperative) -- AC refinement always, AC
// first scans in the pipelined launch.  The lane-per-interval decoder above leaves a batch's
// refinement levels with a few dozen waves on a 1024-SIMD chip (one Y refinement scan per
// image), each lane walking ~10^5 divergent symbols.  Here the wave owns one interval: per window
// step lane l peeks the 32 bits at pos + l and looks its Huffman code up in the wave's LDS table
// (one lookup latency for 64 candidate offsets), then a scalar (SGPR) chain walks the true symbol
// positions through readlane -- the refinement state machine (zero-run targets, EOB runs,
// correction-bit counts on the 64-bit nonzero mask) is SALU work.  The bitstream window (64 + 64
// words), the coming blocks' nonzero masks and the pending records live one per lane in VGPRs;
// records leave 64 blocks at a time (coalesced), one 32-B record per block that k_prog_fold
// applies (its correction bits in walk order, new positions, signs); a first scan's block is assembled
// across the lanes (lane q = coefficient q) and leaves as one masked 16-bit store, exactly the
// halfwords lane_ac_first writes.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t lane) {
  return uint32_t(__builtin_amdgcn_readlane(int(v), int(lane)));
}
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return uint32_t(__builtin_amdgcn_readfirstlane(int(v))); }
// lane `lane` of three 64-bit per-lane values set to the wave-uniform a, b, c (v_writelane: one
// instruction per word, no per-lane compare and selects; the lane select goes through M0 -- two
// SGPR operands would exceed the constant bus -- and the s_nop covers its SALU write)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0: reserved, but nothing else in these kernels uses it
__device__ __forceinline__ void wl64x3(uint64_t &ra, uint64_t &rb, uint64_t &rc, uint64_t a, uint64_t b, uint64_t c,
                                       uint32_t lane) {
  uint32_t a0 = uint32_t(ra), a1 = uint32_t(ra >> 32), b0 = uint32_t(rb), b1 = uint32_t(rb >> 32);
  uint32_t c0 = uint32_t(rc), c1 = uint32_t(rc >> 32);
  asm volatile(
      "s_mov_b32 m0, %12\n\ts_nop 3\n\tv_writelane_b32 %0, %6, m0\n\tv_writelane_b32 %1, %7, m0\n\t"
      "v_writelane_b32 %2, %8, m0\n\tv_writelane_b32 %3, %9, m0\n\tv_writelane_b32 %4, %10, m0\n\t"
      "v_writelane_b32 %5, %11, m0"
      : "+v"(a0), "+v"(a1), "+v"(b0), "+v"(b1), "+v"(c0), "+v"(c1)
      : "s"(uint32_t(a)), "s"(uint32_t(a >> 32)), "s"(uint32_t(b)), "s"(uint32_t(b >> 32)), "s"(uint32_t(c)),
        "s"(uint32_t(c >> 32)), "s"(lane)
      : "m0");
  ra = (uint64_t(a1) << 32) | a0;
  rb = (uint64_t(b1) << 32) | b0;
  rc = (uint64_t(c1) << 32) | c0;
}
#pragma clang diagnostic pop

__global__ __launch_bounds__(64) void k_prog_wave(const RjImageDev *__restrict__ imgs, int nimg,
                                                  const uint32_t *__restrict__ ivals, const uint8_t *__restrict__ destuffed,
                                                  uint32_t *__restrict__ coef, unsigned long long *__restrict__ nz,
                                                  unsigned long long *__restrict__ recs,
                                                  uint32_t *__restrict__ progress, uint32_t progress_n,
                                                  unsigned long long *__restrict__ stamps, uint32_t flags) {
  // development (RJ_DEBUG_WAVES): wall-clock stamps per wave -- start, producers' first window
  // ready, end
  struct WaveStamp {
    unsigned long long *p;
    uint32_t nwin, nstep;
    __device__ ~WaveStamp() {
      if (p && threadIdx.x == 0) {
        *gp(p + 2) = wall_clock64();
        *gp(p + 3) = (uint64_t(nwin) << 32) | nstep;
      }
    }
  } stamp{stamps ? stamps + 4ull * blockIdx.x : nullptr, 0u, 0u};
  if (stamp.p && threadIdx.x == 0) {
    const unsigned long long t = wall_clock64();
    *gp(stamp.p) = t;
    *gp(stamp.p + 1) = t;
  }
  __shared__ uint16_t s_lut[RJ_LUT_ENTRIES];
  __shared__ uint32_t s_maxc[18];
  __shared__ int32_t s_voff[18];
  __shared__ uint8_t s_vals[256];
  const uint32_t lane = threadIdx.x;
  const uint32_t gi = rfl(*gp(ivals + blockIdx.x));
  const int i = int(rfl(uint32_t(upper_index(nimg, gi, [&](int q) { return imgs[q].pival_prefix; }))));
  const RjImageDev &im = imgs[i];
  const RjProgIvalDev iv = *gp(im.pivals + (gi - im.pival_prefix));
  // pipelined launch (progress != null): every refinement interval of the call in one grid, in
  // level order; an interval publishes how many of its units have their records and nonzero
  // masks out, and a later scan's interval waits for its producers' units before it reads masks
  auto publish = [&](uint32_t units_out) {
    if (progress == nullptr) return;
    // mask updates before the count: one release fence (a seq_cst __threadfence would also
    // invalidate the L2), then a relaxed store
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (threadIdx.x == 0) __hip_atomic_store(progress + gi, units_out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  const RjProgScanDev &sc = *gp(im.pscans + iv.scan);
  // The luma AC refinements are the grid's longest chains (one image's final one alone ~43 ms):
  // they issue first on a SIMD they share with other scans' waves (s_setprio; C5 +2.6-3.4 %
  // same-box, profiles/r5_experiments/c5_prio_ab.txt).  RJ_PROG_PRIO_MODE (A/B builds): 0 none,
  // 1 luma refinements, 2 every refinement, 3 graded (luma refinements 3, chroma refinements 2,
  // luma first scans 1), 4 luma refinements 3 and luma first scans 2, 5 every luma scan 3
#ifndef RJ_PROG_PRIO_MODE
#define RJ_PROG_PRIO_MODE 1
#endif
  {
    const uint32_t kind = rfl(uint32_t(sc.kind)), luma = (rfl(uint32_t(sc.comp[0])) & 3u) == 0;
    if (RJ_PROG_PRIO_MODE == 1 && kind == RJ_PK_AC_REFINE && luma) __builtin_amdgcn_s_setprio(3);
    if (RJ_PROG_PRIO_MODE == 2 && kind == RJ_PK_AC_REFINE) __builtin_amdgcn_s_setprio(3);
    if (RJ_PROG_PRIO_MODE == 3) {
      if (kind == RJ_PK_AC_REFINE && luma) __builtin_amdgcn_s_setprio(3);
      else if (kind == RJ_PK_AC_REFINE) __builtin_amdgcn_s_setprio(2);
      else if (luma) __builtin_amdgcn_s_setprio(1);
    }
    if (RJ_PROG_PRIO_MODE == 4 && luma) {
      if (kind == RJ_PK_AC_REFINE) __builtin_amdgcn_s_setprio(3);
      else __builtin_amdgcn_s_setprio(2);
    }
    if (RJ_PROG_PRIO_MODE == 5 && luma) __builtin_amdgcn_s_setprio(3);
  }
  const uint32_t ss = rfl(sc.ss), se = rfl(sc.se);
  const uint64_t band = (se >= 63 ? ~0ull : ((1ull << (se + 1)) - 1)) & ~((1ull << ss) - 1);
  const uint32_t nunits = rfl(iv.nunits), dst_len = rfl(iv.dst_len);
  const uint32_t nbits = dst_len * 8u, nwords = (dst_len + 3) / 4;
  const uint32_t *data = reinterpret_cast<const uint32_t *>(destuffed + im.destuff_off + iv.dst_off);
  const uint32_t c0 = sc.comp[0] & 3u;
  unsigned long long *nzs =
      nz + im.nz_off + (c0 == 0 ? im.nzblk0[0] : (c0 == 1 ? im.nzblk0[1] : im.nzblk0[2])) + iv.unit0;
  const uint32_t nprod = progress ? min(uint32_t(sc.nprod), 3u) : 0u;
  uint32_t *progress_err = progress ? progress + progress_n : nullptr;
  // the last count seen per producer (its interval index, count): units below it need neither a
  // poll nor another acquire fence
  uint32_t seen_j0 = ~0u, seen_j1 = ~0u, seen_j2 = ~0u, seen_n0 = 0, seen_n1 = 0, seen_n2 = 0;
  auto wait_units = [&](uint32_t ub, uint32_t ue) {  // producers' masks of units [ub, ue) are out
    if (ub >= ue) return;
    const uint32_t lo = iv.unit0 + ub, hi = iv.unit0 + ue;
    bool polled = false;
#pragma unroll
    for (uint32_t q = 0; q < 3; q++) {
      if (q >= nprod) break;
      const uint32_t pq = rfl(q == 0 ? sc.prod[0] : (q == 1 ? sc.prod[1] : sc.prod[2]));
      const RjProgScanDev *ps = im.pscans + pq;
      // first scans decoded before this grid: nothing to wait for
      if ((flags & RJ_WAVE_FIRST_DONE) && rfl(gp(ps)->kind) == RJ_PK_AC_FIRST) continue;
      const uint32_t pri = rfl(gp(ps)->ri), pival0 = rfl(gp(ps)->ival0);
      const uint32_t j0 = pri ? lo / pri : 0u, j1 = pri ? (hi - 1) / pri : 0u;
      uint32_t &sj = q == 0 ? seen_j0 : (q == 1 ? seen_j1 : seen_j2);
      uint32_t &sn = q == 0 ? seen_n0 : (q == 1 ? seen_n1 : seen_n2);
      for (uint32_t j = j0; j <= j1; j++) {
        const uint32_t s0 = pri ? j * pri : 0u;
        // units of producer interval j (capped by its DONE); the test hook waits for a count
        // no producer reaches, so that the give-up path runs
        const uint32_t need = (flags & RJ_WAVE_TEST_GIVEUP) ? 0xFFFFFFFEu : hi - s0;
        const uint32_t spin_max = (flags & RJ_WAVE_TEST_GIVEUP) ? 16u : (1u << 23);
        if (j == sj && need <= sn) continue;
        uint32_t *pp = progress + im.pival_prefix + pival0 + j;
        // relaxed polls (an acquire load would invalidate the L2 on every poll), then one acquire
        // fence; bounded (~4 s): a producer that never reports would otherwise hang the GPU --
        // the host turns the flag into EXECUTION_FAILED
        uint32_t got = __hip_atomic_load(pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (uint32_t spin = 0; got < need; spin++) {
          if (spin >= spin_max) {
            if (threadIdx.x == 0) __hip_atomic_store(progress_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          __builtin_amdgcn_s_sleep(8);
          got = __hip_atomic_load(pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        sj = j;
        sn = rfl(got);
        polled = true;
      }
    }
    if (polled) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  };
  auto wait_producers = [&](uint32_t ub) { wait_units(ub, min(ub + 64, nunits)); };
  // a scan's progress stands for its producers' too (a consumer lists only the latest scan of each
  // of its coefficients): an interval reports DONE only once its producers covered all its units
  auto finish = [&](uint32_t ub) {
    wait_units(ub, nunits);
    publish(RJ_PROG_DONE);
  };
  if (iv.flags & RJ_SEG_MISSING) {
    finish(0);
    return;
  }
  const uint32_t kind = rfl(sc.kind);
  // DC first: both tables' first levels (s_lut[0, 512) and [512, 1024)); longer codes are
  // decoded canonically in the chain
  if (kind != RJ_PK_DC_REFINE) {
    const RjHuffDev *gt = im.ptabs + sc.tab[0];
    const uint4 *src = reinterpret_cast<const uint4 *>(gt->lut);
    uint4 *dst = reinterpret_cast<uint4 *>(s_lut);
    if (kind == RJ_PK_DC_FIRST) {
      const RjHuffDev *gt1 = im.ptabs + (sc.tab[1] == 0xFFFFu ? sc.tab[0] : sc.tab[1]);
      dst[lane] = gp(src)[lane];
      dst[64 + lane] = gp(reinterpret_cast<const uint4 *>(gt1->lut))[lane];
    } else {
      for (uint32_t q = lane; q < RJ_LUT_ENTRIES * 2 / 16; q += 64) dst[q] = gp(src)[q];
    }
    if (lane < 18) {
      s_maxc[lane] = gp(gt->maxcode16)[lane];
      s_voff[lane] = gp(gt->valoff)[lane];
    }
    reinterpret_cast<uint32_t *>(s_vals)[lane] = gp(reinterpret_cast<const uint32_t *>(gt->vals))[lane];
  }
  __syncthreads();
  auto ldraw = [&](uint32_t w) -> uint32_t { return *gp(data + min(w, nwords ? nwords - 1 : 0u)); };
  auto cvt = [&](uint32_t w, uint32_t v) -> uint32_t { return w < nwords ? __builtin_bswap32(v) : 0u; };
  auto ldword = [&](uint32_t w) -> uint32_t { return cvt(w, ldraw(w)); };  // zero past the data
  // windows: bitstream words [wbase, wbase + 128) in win0/win1 (lane l: word wbase + l / + 64 + l);
  // the 64 words after them wait unconverted in win2 -- loaded a whole window ahead, so a slide
  // never waits on memory (a wait would also wait for every store the wave has in flight)
  uint32_t wbase = 0;
  uint32_t win0 = ldword(lane), win1 = ldword(64 + lane), win2 = ldraw(128 + lane);
  auto slide = [&]() {
    wbase += 64;
    win0 = win1;
    win1 = cvt(wbase + 64 + lane, win2);
    win2 = ldraw(wbase + 128 + lane);
  };
  auto word = [&](uint32_t w) -> uint32_t {  // w relative to wbase, < 128
    return w < 64 ? rl(win0, w) : rl(win1, w - 64);
  };
  // window step: slide the bitstream window, then 64 candidate decodes -- lane l's 32-bit peek
  // at pos + l and its table entry (len << 8 | r << 4 | s)
  auto candidates = [&](uint32_t pos, uint32_t &pk_l, uint32_t &e_l) {
    if ((pos >> 5) - wbase >= 64) slide();  // everything needed is in win1
    const uint32_t W = (pos >> 5) - wbase, sh = pos & 31;
    const uint32_t A = word(W), B = word(W + 1), C = word(W + 2), D = word(W + 3);
    const uint32_t o = sh + lane;
    const uint32_t hi = o < 32 ? A : (o < 64 ? B : C), lo = o < 32 ? B : (o < 64 ? C : D);
    pk_l = uint32_t(((uint64_t(hi) << 32 | lo) << (o & 31)) >> 32);
    e_l = s_lut[pk_l >> 23];
    if (e_l & 0x8000u) {
      if (e_l == 0xFFFFu) {
        const uint32_t p16 = pk_l >> 16;
        e_l = RJ_LUT_BAD;
        for (int l = 1; l <= 16; l++)
          if (p16 < s_maxc[l]) {
            e_l = uint32_t(l << 8) | s_vals[((p16 >> (16 - l)) + s_voff[l]) & 255];
            break;
          }
      } else {
        e_l = s_lut[RJ_LUT_L1 + (e_l & 0xFFu) * 128u + ((pk_l >> 16) & 127u)];
      }
    }
  };
  if (kind == RJ_PK_DC_REFINE) {
    // ---- DC refinement: the records are the interval's bits, one per block in decode order
    // (lane_dc<true>): record word w = stream bits [64w, 64w + 64), LSB first; zero past the data
    unsigned long long *rec = recs + im.prec_off + iv.rec_off;
    const uint64_t nblocks = uint64_t(nunits) * rfl(sc.nblk);
    const uint32_t nrw = uint32_t((nblocks + 63) / 64);
    for (uint32_t w = lane; w < nrw; w += 64) {
      uint64_t v = __builtin_bitreverse64((uint64_t(ldword(2 * w)) << 32) | ldword(2 * w + 1));
      const uint64_t b0 = uint64_t(w) * 64;
      const uint64_t lim = min(uint64_t(nbits), nblocks);
      v = b0 >= lim ? 0ull : (lim - b0 >= 64 ? v : v & ((1ull << (lim - b0)) - 1));
      *gp(rec + w) = v;
    }
    finish(0);
    return;
  }
  if (kind == RJ_PK_DC_FIRST) {
    // ---- DC first (possibly interleaved): the DC of 64 consecutive blocks collects in the lanes
    // (lane j: block j of the batch) and leaves as 64 halfword stores ----
    const uint32_t al = rfl(sc.al), ns = rfl(sc.ns ? uint32_t(sc.ns) : 1u);
    const uint32_t units_x = rfl(sc.units_x ? uint32_t(sc.units_x) : 1u);
    const uint32_t tsel = rfl(uint32_t(sc.tsel[0]) | (uint32_t(sc.tsel[1]) << 1) | (uint32_t(sc.tsel[2]) << 2));
    uint32_t cbq[3], wbq[3], hsq[3], vsq[3];
#pragma unroll
    for (int q = 0; q < 3; q++) {
      const uint32_t c = sc.comp[q] & 3u;
      cbq[q] = rfl(c == 0 ? im.cblk0[0] : (c == 1 ? im.cblk0[1] : im.cblk0[2]));
      wbq[q] = rfl(c == 0 ? im.wblk[0] : (c == 1 ? im.wblk[1] : im.wblk[2]));
      hsq[q] = rfl(sc.hs[q] ? uint32_t(sc.hs[q]) : 1u);
      vsq[q] = rfl(sc.vs[q] ? uint32_t(sc.vs[q]) : 1u);
    }
    uint16_t *coef16 = reinterpret_cast<uint16_t *>(coef + im.coef_off);
    uint32_t ux = iv.unit0 % units_x, uy = iv.unit0 / units_x;
    uint32_t pos = 0, u = 0, ci = 0, dx = 0, dy = 0, nb = 0, vblk = 0, vval = 0;
    int32_t pred0 = 0, pred1 = 0, pred2 = 0;
    bool done = nunits == 0;
    // codes longer than 9 bits: canonical decode at the true symbol positions only (scalar loads
    // from the table in global memory; rare), not at every candidate offset
    const RjHuffDev *gdc0 = im.ptabs + sc.tab[0];
    const RjHuffDev *gdc1 = im.ptabs + (sc.tab[1] == 0xFFFFu ? sc.tab[0] : sc.tab[1]);
    auto canon = [&](uint32_t p16, const RjHuffDev *g) -> uint32_t {
      for (int l = 1; l <= 16; l++)
        if (p16 < gp(g->maxcode16)[l]) return uint32_t(l << 8) | gp(g->vals)[((p16 >> (16 - l)) + gp(g->valoff)[l]) & 255];
      return RJ_LUT_BAD;
    };
    while (!done) {
      // window step: lane l's peek at pos + l and its entry in both tables
      if ((pos >> 5) - wbase >= 64) slide();
      const uint32_t W = (pos >> 5) - wbase, sh = pos & 31;
      const uint32_t A = word(W), B = word(W + 1), C = word(W + 2), D = word(W + 3);
      const uint32_t o = sh + lane;
      const uint32_t hi = o < 32 ? A : (o < 64 ? B : C), lo = o < 32 ? B : (o < 64 ? C : D);
      const uint32_t pk_l = uint32_t(((uint64_t(hi) << 32 | lo) << (o & 31)) >> 32);
      const uint32_t e0_l = s_lut[pk_l >> 23], e1_l = s_lut[512 + (pk_l >> 23)];
      const uint32_t pos0 = pos;
      while (!done && pos - pos0 < 64) {
        const uint32_t d = pos - pos0;
        const uint32_t t1 = (tsel >> ci) & 1u;
        const uint32_t pk = rl(pk_l, d);
        uint32_t en = t1 ? rl(e1_l, d) : rl(e0_l, d);
        if (en & 0x8000u) en = canon(pk >> 16, t1 ? gdc1 : gdc0);
        const uint32_t len = en >> 8, s = en & 15u;
        const int32_t diff = pextend(pbits(pk, len, s), s);
        int32_t p;
        if (ci == 0) p = pred0 += diff;
        else if (ci == 1) p = pred1 += diff;
        else p = pred2 += diff;
        pos += len + s;
        const uint32_t h = ci == 0 ? hsq[0] : (ci == 1 ? hsq[1] : hsq[2]);
        const uint32_t v = ci == 0 ? vsq[0] : (ci == 1 ? vsq[1] : vsq[2]);
        const uint32_t cb = ci == 0 ? cbq[0] : (ci == 1 ? cbq[1] : cbq[2]);
        const uint32_t wb = ci == 0 ? wbq[0] : (ci == 1 ? wbq[1] : wbq[2]);
        if (lane == nb) {
          vblk = cb + (uy * v + dy) * wb + ux * h + dx;
          vval = uint32_t(p) << al;
        }
        if (++nb == 64) {
          gst16(coef16 + vblk * 64u, vval);
          nb = 0;
        }
        // next slot of the unit
        if (++dx == h) {
          dx = 0;
          if (++dy == v) {
            dy = 0;
            if (++ci == ns) {
              ci = 0;
              u++;
              if (++ux == units_x) {
                ux = 0;
                uy++;
              }
              done = u >= nunits || pos > nbits;
            }
          }
        }
      }
    }
    if (lane < nb) gst16(coef16 + vblk * 64u, vval);
    finish(0);
    return;
  }
  if (kind == RJ_PK_AC_FIRST) {
    // ---- AC first scan: coefficient q of the current block sits in lane q until the block ends ----
    const uint32_t al = rfl(sc.al);
    const uint32_t units_x = rfl(sc.units_x ? uint32_t(sc.units_x) : 1u);
    const uint32_t cb = c0 == 0 ? im.cblk0[0] : (c0 == 1 ? im.cblk0[1] : im.cblk0[2]);
    const uint32_t wb = c0 == 0 ? im.wblk[0] : (c0 == 1 ? im.wblk[1] : im.wblk[2]);
    uint16_t *coef16 = reinterpret_cast<uint16_t *>(coef + im.coef_off);
    uint32_t ux = iv.unit0 % units_x, uy = iv.unit0 / units_x;
    uint32_t pos = 0, k = ss, u = 0, published = 0, cur = 0;
    uint64_t curm = 0;
    bool done = nunits == 0;
    while (!done) {
      uint32_t pk_l, e_l;
      candidates(pos, pk_l, e_l);
      const uint32_t pos0 = pos;
      while (!done && pos - pos0 < 64) {
        const uint32_t d = pos - pos0;
        const uint32_t en = rl(e_l, d);
        const uint32_t len = en >> 8, r = (en >> 4) & 15u, s = en & 15u;
        uint32_t eobrun = 0;
        if (s) {
          const uint32_t q = min(k + r, 63u);
          const int32_t v = pextend(pbits(rl(pk_l, d), len, s), s);
          const uint32_t hv = ((uint32_t(v < 0 ? -v : v) << al) & 0x7FFFu) | (v < 0 ? 0x8000u : 0u);
          if (q <= se) {  // past Se (corrupt data): dropped, as in lane_ac_first
            if (lane == q) cur = hv;
            curm |= 1ull << q;
          }
          k += r + 1;
          pos += len + s;
        } else if (r == 15) {
          k += 16;
          pos += len;
        } else {  // EOBr: this block and eobrun more end here
          eobrun = r ? (1u << r) + pbits(rl(pk_l, d), len, r) - 1u : 0u;
          k = se + 1;
          pos += len + r;
        }
        if (k <= se) continue;
        // ---- block end: its coefficients (one masked halfword store) and nonzero mask ----
        if (curm) {
          const uint32_t blk = cb + uy * wb + ux;
          if ((curm >> lane) & 1u) gst16(coef16 + blk * 64u + lane, cur);
          if (lane == 0) gor64(nzs + u, curm);  // other scans of the component share the word
          curm = 0;
        }
        k = ss;
        const uint32_t step = 1u + min(eobrun, nunits - u - 1u);
        u += step;
        ux += step;
        if (ux >= units_x) {
          uy += ux / units_x;
          ux %= units_x;
        }
        done = u >= nunits || pos > nbits;
        if (done || (u >> 8) != (published >> 8)) {
          publish(done ? RJ_PROG_DONE : u);
          published = u;
        }
      }
    }
    publish(RJ_PROG_DONE);
    return;
  }
  unsigned long long *rec = recs + im.prec_off + iv.rec_off;
  auto ldnz = [&](uint32_t u) -> uint64_t { return *gp(nzs + min(u, nunits - 1)); };
  // nonzero masks of units [nbase, nbase + 64)
  uint32_t nbase = 0;
  if (nunits) wait_producers(0);
  if (stamp.p && threadIdx.x == 0) *gp(stamp.p + 1) = wall_clock64();
  uint64_t nzw = ldnz(lane);
  uint64_t r_cs = 0, r_sg = 0, r_nw = 0;  // lane b: record of unit rbase + b
  uint32_t rbase = 0;
  uint32_t pos = 0, k = ss, eobrun = 0, u = 0;
  uint64_t nzm = uint64_t(rl(uint32_t(nzw), 0)) | (uint64_t(rl(uint32_t(nzw >> 32), 0)) << 32);
  nzm &= band;
  // the block's zero-history positions and, in lane l, how many of them lie below l: the fast
  // path's zero-run target is then the candidate whose rank is (rank of k) + r, one compare
  uint64_t zmb = ~nzm & band;
  uint32_t rank_l = __builtin_amdgcn_mbcnt_hi(uint32_t(zmb >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(zmb), 0u));
  uint64_t cstr = 0, sgn = 0, newm = 0;
  uint32_t pend = 0, t = 0, newv = 0;
  bool walking = false, eobblk = false, done = nunits == 0;
  while (!done) {
    uint32_t pk_l, e_l;
    candidates(pos, pk_l, e_l);
    // per candidate offset, everything that depends only on the bits there (lane-parallel, off
    // the chain): bits used by the symbol and its extra bits, run length r, EOB flag, new
    // value (bit 0: one, bit 1: negative), EOB-run length; and the 32 bits after them (corrections)
    uint32_t info_l, ck_l;
    {
      const uint32_t len = e_l >> 8, r = (e_l >> 4) & 15u, s = e_l & 15u;
      const bool eob = s == 0 && r != 15;
      const uint32_t extra = eob ? r : (s ? 1u : 0u);
      const uint32_t eb = pbits(pk_l, len, extra);
      const uint32_t used = len + extra;
      const uint32_t nv = s ? (eb ? 1u : 3u) : 0u;
      const uint32_t run = eob ? (1u << r) + eb : 0u;
      info_l = used | (r << 6) | (eob ? 1u << 10 : 0u) | (nv << 11) | (run << 13);
      ck_l = used < 32 ? pk_l << used : 0u;
    }
    const uint32_t pos0 = pos;
    stamp.nwin++;
    // ---- scalar chain over the window ----
    while (!done && pos - pos0 < 64) {
#ifndef RJ_PW_NO_FAST
      // ---- fast path: the common symbol (no EOB, no pending walk, its correction bits inside
      // this peek, the block not ending with it), as a tight loop with none of the rare state
      // live; anything else leaves it with the symbol unconsumed for the general step below,
      // which decodes it exactly as it would have ----
      if (__builtin_expect(!walking && eobrun == 0, 1)) {
        __builtin_assume(k < 64u);
        // zero-history positions below k; inside the loop it follows the target: k = tf + 1
        uint32_t rk = uint32_t(__popcll(zmb & ~(~0ull << k)));
        const uint64_t zmf = zmb & ~(1ull << se);
        for (;;) {
          const uint32_t df = pos - pos0;
          if (df >= 64) break;
          const uint32_t info = rl(info_l, df);
          if (info & (1u << 10)) break;  // EOBr
          const uint32_t r = (info >> 6) & 15u, usedf = info & 63u;
          // the (r+1)-th zero-history position at or after k: rank rk + r (a lane of lower rank
          // in zmb lies below k; none of another rank can match); the lanes' rank relative to k
          // is formed off the symbol's readlane
          const uint32_t rel = rank_l - rk;
          // (zmf: without Se -- a target at Se, or none, ends the block: the general step)
          const uint64_t hit = __ballot(rel == r) & zmf;
          if (!hit) break;
          uint32_t tf;
          asm("s_ff1_i32_b64 %0, %1" : "=s"(tf) : "s"(hit));
          // [k, tf) holds r zero-history positions; the others take a correction bit each
          const uint32_t pf = (tf - k) - r;
          if (usedf + pf > 32u) break;  // the walk crosses into the next peek
          const uint32_t cb = rl(ck_l, df);
          cstr = (cstr << pf) | uint32_t((uint64_t(cb) << pf) >> 32);
          pos += usedf + pf;
          // tf < se <= 63 here; a new coefficient's bit and its sign bit, shifted into place
          __builtin_assume(tf < 64u);
          newm |= uint64_t((info >> 11) & 1u) << tf;
          sgn |= uint64_t((info >> 12) & 1u) << tf;
          k = tf + 1;
          rk += r + 1u;
        }
        if (pos - pos0 >= 64) continue;  // the window is used up: the next one
      }
#endif
      const uint32_t d = pos - pos0;
      stamp.nstep++;
      uint32_t used = 0, cbits;
      if (__builtin_expect(!walking, 1)) {  // (hints: the common symbol falls through)
        if (__builtin_expect(eobrun == 0, 1)) {
          const uint32_t info = rl(info_l, d);
          cbits = rl(ck_l, d);
          const uint32_t r = (info >> 6) & 15u;
          used = info & 63u;
          if (__builtin_expect(!(info & (1u << 10)), 1)) {
            newv = (info >> 11) & 3u;
            // the (r+1)-th zero-history position at or after k, lane-parallel: lane l is it when
            // bit l of the candidate mask is set with exactly r candidates below it
            __builtin_assume(k < 64u);
            const uint64_t zm = ~nzm & band & (~0ull << k);
            const uint32_t below =
                __builtin_amdgcn_mbcnt_hi(uint32_t(zm >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(zm), 0u));
            // the lanes with exactly r candidates below them, masked by the candidates on the
            // SALU (a ballot of the compare alone: no per-lane bit test)
            const uint64_t hit = __ballot(below == r) & zm;
            t = hit ? ctz64(hit) : se + 1;
            // [k, t) lies in the band: r of its positions have zero history (every candidate when
            // nothing hit), the others take one correction bit each
            pend = (t - k) - min(r, uint32_t(__popcll(zm)));
            eobblk = false;
          } else {  // EOBr
            eobrun = rfl(info >> 13);
            t = se + 1;
            newv = 0;
            eobblk = true;
            __builtin_assume(k < 64u);
            pend = uint32_t(__popcll(nzm & (~0ull << k)));
          }
        } else {  // a block inside an EOB run
          cbits = rl(pk_l, d);
          t = se + 1;
          newv = 0;
          eobblk = true;
          __builtin_assume(k < 64u);
          pend = uint32_t(__popcll(nzm & (~0ull << k)));
        }
        walking = true;
      } else {
        cbits = rl(pk_l, d);
      }
      const uint32_t take = min(pend, 32u - used);
      // the top `take` bits of cbits (none for take = 0): the high word of a 64-bit shift
      cstr = (cstr << take) | uint32_t((uint64_t(cbits) << take) >> 32);
      used += take;
      pend -= take;
      pos += used;
      if (__builtin_expect(pend != 0, 0)) continue;  // the walk resumes at the next peek
      walking = false;
      // a new coefficient whose zero run overshoots the band (corrupt data): at Se = 63 libjpeg
      // stores it at natural position 63 (jpeg_natural_order[64] == 63, oracle kZigzag[64]);
      // past a smaller Se it is dropped (see lane_ac_first)
      const uint32_t tc = min(t, 63u);
      if (newv && tc <= se) {
        __builtin_assume(tc < 64u);
        const uint64_t bq = 1ull << tc;
        newm |= bq;
        sgn |= newv == 3 ? bq : 0ull;
      }
      bool blk_done;
      if (__builtin_expect(eobblk, 0)) {
        eobrun = rfl(eobrun - 1u);
        blk_done = true;
      } else {
        k = t + 1;
        blk_done = k > se;
      }
      if (__builtin_expect(!blk_done, 1)) continue;
      // ---- block end: its record into lane (u - rbase); 64 records leave together ----
      const uint32_t rb = u - rbase;
      // into lane rb by v_writelane (one instruction per word, no per-lane compare and selects)
      wl64x3(r_cs, r_sg, r_nw, cstr, sgn, newm, rb);
      cstr = sgn = newm = 0;
      k = ss;
      u++;
      done = u >= nunits || pos > nbits;
      if (rb == 63 || done) {
        if (rbase + lane < u) {
          uint4 *r4 = reinterpret_cast<uint4 *>(rec + uint64_t(rbase + lane) * 4u);
          *gp(r4) = make_uint4(uint32_t(r_cs), uint32_t(r_cs >> 32), uint32_t(r_sg), uint32_t(r_sg >> 32));
          *gp(r4 + 1) = make_uint4(uint32_t(r_nw), uint32_t(r_nw >> 32), 0u, 0u);
          // the new nonzero positions go to the masks now (other scans of this level may share
          // the word: atomic); k_prog_fold peels them again where it needs the earlier state
          if (r_nw) gor64(nzs + rbase + lane, r_nw);
        }
        if (done) finish(nbase);
        else if ((u & 255u) == 0) publish(u);  // every 256 units: fewer release fences
        r_cs = r_sg = r_nw = 0;
        rbase += 64;
      }
      if (done) break;
      if (u - nbase >= 64) {
        nbase += 64;
        wait_producers(nbase);
        nzw = ldnz(nbase + lane);
      }
      const uint32_t nl = u - nbase;
      nzm = (uint64_t(rl(uint32_t(nzw), nl)) | (uint64_t(rl(uint32_t(nzw >> 32), nl)) << 32)) & band;
      zmb = ~nzm & band;
      rank_l = __builtin_amdgcn_mbcnt_hi(uint32_t(zmb >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(zmb), 0u));
    }
  }
  finish(nbase);  // every exit (an empty interval never flushed)
}

hipError_t LaunchProgressiveWave(hipStream_t st, const RjImageDev *imgs, int nimg, const uint32_t *ivals, uint32_t n,
                                 const uint8_t *destuffed, uint32_t *coef, unsigned long long *nz,
                                 unsigned long long *recs, uint32_t *progress, uint32_t progress_n,
                                 unsigned long long *stamps, uint32_t flags) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_prog_wave, dim3(n), dim3(64), 0, st, imgs, nimg, ivals, destuffed, coef, nz, recs, progress,
                     progress_n, stamps, flags);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// k_prog_fold: a dependency level's refinement records into the dense coefficients and the
// nonzero masks.  One lane per block of one component of one image (a wave = 64 blocks of one
// job, so the job and the image's scan list are wave-uniform); every block is owned by one lane,
// so the read-modify-write needs no atomics.  All updates are ORs: AC magnitude bit Al (and the
// sign of a new coefficient), DC bit Al (libjpeg decode_mcu_DC_refine: block[0] |= p1).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void or_bits(uint32_t (&w)[32], uint64_t orm, uint64_t sgn, uint32_t p1) {
#pragma unroll
  for (int q = 0; q < 32; q++) {
    const uint32_t m2 = uint32_t(orm >> (2 * q)) & 3u, s2 = uint32_t(sgn >> (2 * q)) & 3u;
    w[q] |= ((m2 & 1u) ? p1 : 0u) | ((m2 & 2u) ? (p1 << 16) : 0u) | ((s2 & 1u) << 15) | ((s2 & 2u) << 30);
  }
}

__global__ __launch_bounds__(64) void k_prog_fold(const RjImageDev *__restrict__ imgs, const RjFoldJob *__restrict__ jobs,
                                                  uint32_t njobs, uint32_t level, uint32_t *__restrict__ coef,
                                                  unsigned long long *__restrict__ nz,
                                                  const unsigned long long *__restrict__ recs) {
  const uint32_t chunk = blockIdx.x;
  const int j = __builtin_amdgcn_readfirstlane(upper_index(int(njobs), chunk, [&](int q) { return jobs[q].chunk0; }));
  const RjFoldJob J = jobs[j];
  const uint32_t b = (chunk - J.chunk0) * 64u + threadIdx.x;
  if (b >= J.nblocks) return;
  const RjImageDev &im = imgs[J.image];
  const uint32_t c = J.comp;
  const uint32_t wb = c == 0 ? im.wblk[0] : (c == 1 ? im.wblk[1] : im.wblk[2]);
  const uint32_t cwb = c == 0 ? im.cwblk[0] : (c == 1 ? im.cwblk[1] : im.cwblk[2]);
  const uint32_t chb = c == 0 ? im.chblk[0] : (c == 1 ? im.chblk[1] : im.chblk[2]);
  const uint32_t cb0 = c == 0 ? im.cblk0[0] : (c == 1 ? im.cblk0[1] : im.cblk0[2]);
  const uint32_t nzb0 = c == 0 ? im.nzblk0[0] : (c == 1 ? im.nzblk0[1] : im.nzblk0[2]);
  const uint32_t by = b / wb, bx = b - by * wb;
  const bool coded = bx < cwb && by < chb;  // blocks a non-interleaved scan codes
  const unsigned long long *rec = recs + im.prec_off;
  uint32_t w[32];
  bool loaded = false;
  uint4 *blk4 = reinterpret_cast<uint4 *>(coef + im.coef_off + uint64_t(cb0 + b) * 32u);
  auto load = [&]() {
    if (loaded) return;
    loaded = true;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint4 v = gp(blk4)[q];
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
  };
  // the masks already hold every new position of the scans folded here (k_prog_wave ORs them
  // in); walking the scans backwards and peeling each scan's new positions gives the masks each
  // scan saw when it decoded
  const unsigned long long *nzp = nz + im.nz_off + nzb0 + by * cwb + bx;
  uint64_t running = coded ? *gp(nzp) : 0ull;
  const uint32_t ns_img = im.npscans;
  for (uint32_t sr = ns_img; sr-- > 0;) {
    const uint32_t si = sr;
    const RjProgScanDev sc = im.pscans[si];
    if (level != RJ_FOLD_ALL && sc.level != level) continue;
    if (sc.kind == RJ_PK_AC_REFINE) {
      if (sc.comp[0] != c || !coded) continue;
      const uint32_t unit = by * cwb + bx;
      const RjProgIvalDev iv = *gp(im.pivals + sc.ival0 + (sc.ri ? unit / sc.ri : 0u));
      const uint4 *r4 = reinterpret_cast<const uint4 *>(rec + iv.rec_off + uint64_t(unit - iv.unit0) * 4u);
      const uint4 a = *gp(r4), n = *gp(r4 + 1);
      const uint64_t cstr = uint64_t(a.y) << 32 | a.x, sgn = uint64_t(a.w) << 32 | a.z;
      const uint64_t newm = uint64_t(n.y) << 32 | n.x;
      if (cstr | newm) {
        // the correction bits belong to the band's previously nonzero positions, ascending,
        // first bit most significant (libjpeg decode_mcu_AC_refine's walk order)
        const uint64_t band = (sc.se >= 63 ? ~0ull : ((1ull << (sc.se + 1)) - 1)) & ~((1ull << sc.ss) - 1);
        running &= ~newm;
        uint64_t nzm = running & band;
        uint32_t j = uint32_t(__popcll(nzm));
        uint64_t orm = newm;
        while (nzm) {
          const uint32_t q = uint32_t(__builtin_ctzll(nzm));
          nzm &= nzm - 1;
          j--;
          if ((cstr >> j) & 1u) orm |= 1ull << q;
        }
        load();
        or_bits(w, orm, sgn, 1u << sc.al);
      }
    } else if (sc.kind == RJ_PK_DC_REFINE) {
      uint32_t i = 3, slot0 = 0;
      for (uint32_t q = 0; q < sc.ns; q++) {
        if (sc.comp[q] == c && i == 3) i = q;
        if (i == 3) slot0 += uint32_t(sc.hs[q]) * sc.vs[q];
      }
      if (i == 3) continue;
      uint32_t unit, slot;
      if (sc.ns > 1) {
        const uint32_t h = sc.hs[i], v = sc.vs[i];
        const uint32_t mx = bx / h, my = by / v;
        unit = my * sc.units_x + mx;
        slot = slot0 + (by - my * v) * h + (bx - mx * h);
      } else {
        if (!coded) continue;
        unit = by * cwb + bx;
        slot = 0;
      }
      const RjProgIvalDev iv = *gp(im.pivals + sc.ival0 + (sc.ri ? unit / sc.ri : 0u));
      const uint32_t bit = (unit - iv.unit0) * sc.nblk + slot;
      const uint64_t word = *gp(rec + iv.rec_off + bit / 64u);
      if ((word >> (bit & 63u)) & 1u) {
        load();
        w[0] |= 1u << sc.al;  // two's complement DC: bit Al, low half
      }
    }
  }
  if (loaded) {
#pragma unroll
    for (int q = 0; q < 8; q++) gp(blk4)[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  }

}

hipError_t LaunchProgressiveFold(hipStream_t st, const RjImageDev *imgs, const RjFoldJob *jobs, uint32_t njobs,
                                 uint32_t nchunks, uint32_t level, uint32_t *coef, unsigned long long *nz,
                                 const unsigned long long *recs) {
  if (nchunks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_prog_fold, dim3(nchunks), dim3(64), 0, st, imgs, jobs, njobs, level, coef, nz, recs);
  return hipGetLastError();
}

}  // namespace rj
