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
// (9 bits; DC first: two 8-bit tables) in a lane-interleaved LDS column, the bitstream in a
// 32-word LDS ring, and (AC refinement) the nonzero masks of the coming blocks in a 32-entry LDS
// ring.  Both rings are topped up at wave-uniform phase boundaries with loads issued one phase
// before they are committed; the symbol loop itself reads no HBM.
#include <hip/hip_runtime.h>

#include "rj_device.h"
#include "rj_kernels.h"
#include "rj_math.h"

namespace rj {

#define RJ_PW 64       // one wave per workgroup
#define RJ_PPHASE 8    // iterations per phase; an iteration consumes <= 32 bits and <= 1 block
#define RJ_PRING 32    // bit ring words per lane
#define RJ_PNZ 32      // nonzero-mask ring entries per lane

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

// canonical search (second-level pool exhausted): libjpeg jpeg_huff_decode on the HBM table
__device__ __forceinline__ uint32_t phuff_slow(const RjHuffDev *t, uint32_t peek16) {
  uint32_t e = RJ_LUT_BAD;
#pragma unroll 1
  for (int l = 1; l <= 16; l++)
    if (peek16 < gp(t->maxcode16)[l]) {
      e = uint32_t(l << 8) | gp(t->vals)[((peek16 >> (16 - l)) + gp(t->valoff)[l]) & 255];
      break;
    }
  return e;
}
// full two-level lookup in HBM (codes longer than the LDS level resolves)
__device__ __forceinline__ uint32_t phuff_global(const RjHuffDev *t, uint32_t peek) {
  uint32_t e = gp(t->lut)[peek >> 23];
  if (e & 0x8000u) {
    if (e == 0xFFFFu) e = phuff_slow(t, peek >> 16);
    else e = gp(t->lut)[RJ_LUT_L1 + (e & 0xFFu) * 128u + ((peek >> 16) & 127u)];
  }
  return e;
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
__device__ void lane_dc(const PLaneIn &L, PGeo &g, PBits &br, const HRow &lut, uint16_t *coef16, uint32_t *coef32) {
  const RjProgScanDev &sc = L.sc;
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
  const uint32_t al = sc.al;
  const uint32_t tsel = uint32_t(sc.tsel[0]) | (uint32_t(sc.tsel[1]) << 1) | (uint32_t(sc.tsel[2]) << 2);
  const uint32_t nbits = L.iv.dst_len * 8u;
  int32_t pred0 = 0, pred1 = 0, pred2 = 0;
  uint32_t ci = 0, dx = 0, dy = 0;
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
        if (peek >> 31) gor32(coef32 + g.coef + blk * 32u, 1u << al);
        br.pos += 1;
      } else {
        const uint32_t t = (tsel >> ci) & 1u;
        uint32_t e = lut[(t << 8) | (peek >> 24)];
        if (e & 0x8000u) e = phuff_global(t ? gt1 : gt0, peek);
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
            if (g.u >= g.nunits || br.pos > nbits) active = false;
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
__device__ void lane_ac_first(const PLaneIn &L, PGeo &g, PBits &br, const HRow &lut, uint16_t *coef16,
                              unsigned long long *nz, uint32_t nzbase) {
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
      if (e & 0x8000u) e = phuff_global(gt, peek);
      const uint32_t len = e >> 8, r = (e >> 4) & 15u, s = e & 15u;
      if (s) {
        const uint32_t q = min(k + r, 63u);
        const int32_t v = pextend(pbits(peek, len, s), s);
        const uint32_t mag = (uint32_t(v < 0 ? -v : v) << al) & 0x7FFFu;
        const uint32_t blk = pblock(g, 0, 0, 0);
        gst16(coef16 + (g.coef + blk * 32u) * 2u + q, mag | (v < 0 ? 0x8000u : 0u));
        blk_nz |= 1ull << q;
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

__device__ void lane_ac_refine(const PLaneIn &L, PGeo &g, PBits &br, const HRow &lut, uint32_t *coef32,
                               unsigned long long *nz, uint32_t nzbase, PRow nzr) {
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
  const uint32_t ss = sc.ss, se = sc.se, al = sc.al;
  const uint32_t p1 = 1u << al;
  const uint64_t band = lomask(se + 1) & ~lomask(ss);
  const uint32_t nbits = L.iv.dst_len * 8u;
  // nonzero-mask ring: masks of units [0, ntop) relative to the interval are committed
  const unsigned long long *nzsrc = nz + nzbase;
  const uint32_t nlast = g.nunits ? g.nunits - 1 : 0u;
  uint32_t ntop = 0;
  auto nz_put = [&](const uint2 &m) {
    nzr[2 * (ntop & (RJ_PNZ - 1))] = m.x;
    nzr[2 * (ntop & (RJ_PNZ - 1)) + 1] = m.y;
    ntop++;
  };
  {
    uint2 m[24];
#pragma unroll
    for (uint32_t q = 0; q < 24; q++) m[q] = *gp(reinterpret_cast<const uint2 *>(nzsrc + min(q, nlast)));
#pragma unroll
    for (int q = 0; q < 24; q++) nz_put(m[q]);
  }
  uint32_t urel = 0;  // unit relative to the interval (ring index)
  auto nz_get = [&](uint32_t ur) {
    const uint32_t sl = ur & (RJ_PNZ - 1);
    return (uint64_t(nzr[2 * sl + 1]) << 32) | nzr[2 * sl];
  };
  uint64_t nzm = nz_get(0) & band;
  uint32_t k = ss, eobrun = 0, t = 0, newv = 0;
  bool walking = false, eobblk = false;
  uint64_t blk_new = 0;
  bool active = L.active;
  while (__any(active)) {
    uint4 pa, pb;
    const bool rb = br.room();
    br.issue(pa, pb);
    uint2 pm[8];
    const bool rn = ntop + 8 - urel <= RJ_PNZ;
#pragma unroll
    for (uint32_t q = 0; q < 8; q++) pm[q] = *gp(reinterpret_cast<const uint2 *>(nzsrc + min(ntop + q, nlast)));
#pragma unroll 1
    for (int it = 0; it < RJ_PPHASE; it++) {
      if (!active) continue;
      const uint32_t peek = br.peek();
      uint32_t used = 0;
      if (!walking) {
        if (eobrun) {
          t = se + 1;
          newv = 0;
          eobblk = true;
        } else {
          uint32_t e = lut[peek >> 23];
          if (e & 0x8000u) e = phuff_global(gt, peek);
          const uint32_t len = e >> 8, r = (e >> 4) & 15u, s = e & 15u;
          used = len;
          if (s || r == 15) {
            if (s) {
              newv = pbits(peek, used, 1) ? p1 : (0x8000u | p1);
              used++;
            } else {
              newv = 0;
            }
            // the (r+1)-th not-yet-nonzero position at or after k (libjpeg's zero-run walk)
            uint64_t z = ~nzm & band & ~lomask(k);
            for (uint32_t j = 0; j < r; j++) z &= z - 1;
            t = z ? ctz64(z) : se + 1;
          } else {  // EOBr: this block's rest and 2^r + bits - 1 more blocks
            eobrun = (1u << r) + pbits(peek, used, r);
            used += r;
            t = se + 1;
            newv = 0;
            eobblk = true;
          }
        }
        walking = true;
      }
      // correction bits of the nonzero positions in [k, t), at most 32 - used of them
      uint64_t cm = nzm & lomask(t) & ~lomask(k);
      const uint32_t cnt = uint32_t(__popcll(cm));
      const uint32_t take = min(cnt, 32u - used);
      const uint32_t cbits = pbits(peek, used, take);
      used += take;
      const uint32_t dwb = g.coef + pblock(g, 0, 0, 0) * 32u;
      uint32_t lastq = k;
      for (uint32_t j = 0; j < take; j++) {
        const uint32_t q = ctz64(cm);
        cm &= cm - 1;
        if ((cbits >> (take - 1 - j)) & 1u) gor32(coef32 + dwb + (q >> 1), p1 << ((q & 1u) * 16u));
        lastq = q;
      }
      br.pos += used;
      bool blk_done = false;
      if (take < cnt) {
        k = lastq + 1;  // the walk continues next iteration
      } else {
        walking = false;
        if (newv) {
          const uint32_t q = min(t, 63u);
          gor32(coef32 + dwb + (q >> 1), newv << ((q & 1u) * 16u));
          blk_new |= 1ull << q;
        }
        if (eobblk) {
          eobblk = false;
          eobrun--;
          blk_done = true;
        } else {
          k = t + 1;
          blk_done = k > se;
        }
      }
      if (blk_done) {
        if (blk_new) gor64(nz + nzbase + g.u, blk_new);
        blk_new = 0;
        k = ss;
        unit_step(g, 1);
        urel++;
        if (g.u >= g.nunits || br.pos > nbits) active = false;
        else nzm = nz_get(urel) & band;
      }
    }
    br.commit(pa, pb, rb);
    if (rn) {
#pragma unroll
      for (int q = 0; q < 8; q++) nz_put(pm[q]);
    }
  }
}

__global__ __launch_bounds__(RJ_PW) void k_prog(const RjImageDev *__restrict__ imgs, int nimg,
                                                const uint32_t *__restrict__ lanes, uint32_t nlanes,
                                                const uint8_t *__restrict__ destuffed, uint32_t *__restrict__ coef,
                                                unsigned long long *__restrict__ nz) {
  __shared__ uint16_t s_lut[RJ_LUT_L1 * RJ_PW];
  __shared__ uint32_t s_ring[RJ_PRING * RJ_PW];
  __shared__ uint32_t s_nz[2 * RJ_PNZ * RJ_PW];
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

  PBits br;
  const uint8_t *data = L.active ? destuffed + im.destuff_off + L.iv.dst_off : destuffed;
  br.init(reinterpret_cast<const uint4 *>(data), PRow{s_ring + lane}, L.active ? L.iv.dst_len : 0u);
  const HRow lut{s_lut + lane};
  switch (kind) {
    case RJ_PK_DC_FIRST:
      lane_dc<false>(L, g, br, lut, coef16, coef32);
      break;
    case RJ_PK_DC_REFINE:
      lane_dc<true>(L, g, br, lut, coef16, coef32);
      break;
    case RJ_PK_AC_FIRST:
      lane_ac_first(L, g, br, lut, coef16, nzi, nzbase);
      break;
    default:
      lane_ac_refine(L, g, br, lut, coef32, nzi, nzbase, PRow{s_nz + lane});
      break;
  }
}

hipError_t LaunchProgressive(hipStream_t st, const RjImageDev *imgs, int nimg, const uint32_t *lanes, uint32_t nlanes,
                             const uint8_t *destuffed, uint32_t *coef, unsigned long long *nz) {
  if (nlanes == 0) return hipSuccess;
  hipLaunchKernelGGL(k_prog, dim3((nlanes + RJ_PW - 1) / RJ_PW), dim3(RJ_PW), 0, st, imgs, nimg, lanes, nlanes,
                     destuffed, coef, nz);
  return hipGetLastError();
}

}  // namespace rj
