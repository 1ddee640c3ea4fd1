// rj_huff.hip -- K1: baseline Huffman decode (T.81 F.2.2, libjpeg jdhuff.c semantics).
//   k_huff        the lean launch for "row" images (every restart interval inside one MCU row),
//                 one lane per interval (and, for outlier intervals, a head + tail lane pair);
//   k_huff_chunk  every other call: rj_entropy.hip's chunk layout (one lane per chunk of a split
//                 interval, one per whole interval otherwise), records and resolution.
//
// The reference hands this step to VCN (src/rocjpeg_vaapi_decoder.cpp:677-689).  At ~1 wave per
// SIMD (a C2 batch has 68 intervals per image) the serial symbol chain is issue-bound, so the
// step keeps only what the bit position depends on:
//   * one 32-bit table entry per code prefix carries every field the step uses (rj_device.h
//     RjLeanTables): bit count, extra-bit width, run -- and, where it fits the key, the code
//     that follows with its own fields (two symbols per step);
//   * the entry written per coefficient is its HUFF_EXTENDed value and zigzag position; the DC
//     is a difference in the lean launch (K2, rj_fused.hip, restores the predictions for 64
//     blocks at once) and absolute in the chunk launch (the lane keeps libjpeg's predictors);
//   * bits: the two stream words holding the bit position in registers, the next one read one
//     step ahead from the lane's LDS ring, which a mover wave beside each decoder wave keeps
//     filled; a 32-bit peek is one v_alignbit_b32 (q = -pos);
//   * addresses: table bases are LDS byte addresses (a lookup is a shift and a shift-add), the
//     stage and the ring are aligned to their own size (a word's address is one v_and_or_b32),
//     extra bits and their mask are v_bfe_u32s;
//   * block / MCU bookkeeping: the block index inside the MCU selects the tables through a
//     2-bit-per-block pattern; the step is software-pipelined (the next lookup is issued before
//     this symbol's entry is written).
// Everything else (stage flushes, libjpeg's insufficient-data and missing-marker rules, the
// chunk lanes' records and sync tests) happens at wave-uniform phase boundaries every
// RJ_HL_PHASE steps, or only in the phases where some lane may finish or stop.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "rj_device.h"
#include "rj_kernels.h"
#include "rj_math.h"

namespace rj {

#define RJ_HL_CHUNKS 8                      // 16-B chunks in a lane's bit ring
#define RJ_HL_WORDS (RJ_HL_CHUNKS * 4)      // 32 words
#ifndef RJ_HL_PHASE
#define RJ_HL_PHASE 8                       // steps (1-2 symbols each) per phase of the whole-interval launch
#endif
#define RJ_HL_GROUP 16                      // entries per flush group (RJ_ENT_GROUP)
// LDS byte offsets of the four tables (RjLeanTables order)
#define RJ_HL_AC_BYTES (RJ_HL_AC_WORDS * 4)
#define RJ_HL_DC0 (2 * RJ_HL_AC_BYTES)
#define RJ_HL_LUT_WORDS (2 * RJ_HL_AC_WORDS + 2 * RJ_HL_DC_WORDS)
// Split launch (rj_kernels.h LaunchHuffLanes): MCU-start records kept by a tail lane (two
// workgroups per CU must fit in LDS; a head that finds no equal MCU start among them decodes the
// whole interval)
#define RJ_HL_REC 20
#define RJ_HL_REC_LIMIT 65280u              // records are 16-bit bit positions past the split

__device__ const uint4 rj_hl_zero[2] = {};

#ifdef RJ_HL_STAMPS  // diagnostic build: cycles in the symbol steps / the phase ends, summed over waves
__device__ unsigned long long rj_hl_stamp[11];  // [8]: s_memrealtime ticks of the loops (100 MHz), [9] to the flush's end, [10] ring checks
// k_huff_chunk: per decoder wave, summed: setup cycles (entry to the first phase), loop cycles,
// phases, safe phases, waves; max loop cycles; ring-wait cycles
__device__ unsigned long long rj_hc_stamp[14];
#define RJ_HL_COUNT_ESC st_esc++
#else
#define RJ_HL_COUNT_ESC
#endif

// word w of the lane's column of a lane-interleaved LDS array ([w][lane], S lanes: conflict-free)
template <int S>
struct HCol {
  uint32_t *base;
  __device__ __forceinline__ uint32_t &operator[](uint32_t w) const { return base[w * S]; }
};

template <int S>
__device__ __forceinline__ void hl_put(const HCol<S> &ring, uint32_t slot, const uint4 &v) {
  const uint32_t w0 = __builtin_bswap32(v.x), w1 = __builtin_bswap32(v.y);
  const uint32_t w2 = __builtin_bswap32(v.z), w3 = __builtin_bswap32(v.w);
  ring[4 * slot] = w0;
  ring[4 * slot + 1] = w1;
  ring[4 * slot + 2] = w2;
  ring[4 * slot + 3] = w3;
}

// the group of G staged entries [from, from + G) (from a multiple of G; the stage holds 2G) to HBM
template <int S, int G>
__device__ __forceinline__ void hl_flush(const HCol<S> &stage, uint32_t from, uint32_t *dst) {
#ifdef RJ_EXP_NOENT  // timing build (with RJ_EXP_SKIP_K2): K1 writes no entries -- its time without the intermediate
  return;
#endif
  uint32_t w[G];
  const uint32_t s0 = from & (2 * G - 1);
#pragma unroll
  for (int q = 0; q < G; q++) w[q] = stage[s0 + q];
#ifdef RJ_EXP_HALFSTORE  // timing build: the entries' low halves packed in pairs (half the store bytes)
  {
    uint32_t h[G / 2];
#pragma unroll
    for (int q = 0; q < G / 2; q++) h[q] = __builtin_amdgcn_perm(w[2 * q + 1], w[2 * q], 0x05040100u);
    uint4 *d4 = reinterpret_cast<uint4 *>(dst);
#pragma unroll
    for (int q = 0; q < G / 8; q++) gp(d4)[q] = make_uint4(h[4 * q], h[4 * q + 1], h[4 * q + 2], h[4 * q + 3]);
    return;
  }
#endif
#ifdef RJ_EXP_NOSTORE  // timing build: the stage is read, nothing is stored
  if (w[0] == 0x12345678u && w[G - 1] == 0x9ABCDEF0u) *gp(dst) = w[1];
  return;
#endif
#ifdef RJ_EXP_E16  // timing probe (lean calls only): 16-bit entries, position 6 b | value 10 b
  {                 // (clamped: wrong pixels where |value| > 511); -512 marks TERM (pos 63) / ZERO
    uint32_t h[G / 2];
#pragma unroll
    for (int q = 0; q < G; q++) {
      const uint32_t e = w[q], pos = (e >> 16) & 127u;
      const int32_t v = min(max(int32_t(int16_t(e & 0xFFFFu)), -511), 511);
      uint32_t x = (pos << 10) | (uint32_t(v) & 0x3FFu);
      x = (e & (1u << 23)) ? 0x200u : x;
      x = pos == 127u ? ((63u << 10) | 0x200u) : x;
      if (q & 1) h[q / 2] |= x << 16;
      else h[q / 2] = x;
    }
    uint4 *d4 = reinterpret_cast<uint4 *>(dst);
#pragma unroll
    for (int q = 0; q < G / 8; q++) gp(d4)[q] = make_uint4(h[4 * q], h[4 * q + 1], h[4 * q + 2], h[4 * q + 3]);
    return;
  }
#endif
  uint4 *d4 = reinterpret_cast<uint4 *>(dst);
#pragma unroll
  for (int q = 0; q < G / 4; q++) gp(d4)[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

// Codes the first level does not resolve (rare): AC second level, or libjpeg's canonical
// search (jpeg_huff_decode) on the table in HBM, repacked into the entry format (one symbol).
__device__ __forceinline__ uint32_t hl_escape(uint32_t e, uint32_t peek, bool isdc, uint32_t acbase,
                                           const uint32_t *s_lut, const RjTableSet *ts, uint32_t ids) {
  const uint32_t sub = e & 0xFFu;
  const RjHuffDev *t = isdc ? &ts->dc[ids & 1u] : &ts->ac[(ids >> 1) & 1u];
  if (!isdc && sub < RJ_HL_SUBS)
    return s_lut[(acbase >> 2) + (1u << RJ_HL_AC_BITS) + sub * 32u + ((peek >> (32 - RJ_HL_AC_BITS - 5)) & 31u)];
  const uint32_t p16 = peek >> 16;
  uint32_t len = 17, sym = 0;  // bad code: 17 bits, symbol 0 (libjpeg JWRN_HUFF_BAD_CODE)
#pragma unroll 1
  for (uint32_t l = 1; l <= 16; l++)
    if (p16 < t->maxcode16[l]) {
      len = l;
      sym = t->vals[((p16 >> (16 - l)) + t->valoff[l]) & 255];
      break;
    }
  const uint32_t s = sym & 15u, r = sym >> 4;
  const uint32_t R = isdc ? 0u : (s ? r : (r == 15 ? 15u : 63u));
  return ((len + s) << 16) | (s << 21) | (R << 25);
}

// One symbol step -- one or two symbols (rj_device.h RjLeanTables: a table entry may carry the
// code that follows the first one, when both lie inside the first-level key).  SAFE: per-lane
// activity (blocks_left) and libjpeg's insufficient-data rule.  SYNC (split launch): the lane
// notes where its last MCU started (mpos, mleft), and a tail lane records its MCU starts (recs,
// nr; head lanes keep nr = RJ_HL_REC and write a scratch slot).  A block ends at most once per
// step (the second symbol is taken only when the first leaves the block open), so MCU starts,
// the insufficient-data rule and the records see the same block boundaries as one symbol per
// step would.
// Software-pipelined: a step starts with this symbol's entry `e` and its 32-bit `peek` already
// loaded (by the previous step, or the prologue); it first advances the bit position and the
// block / table state -- the chain the next lookup depends on -- and issues the next symbol's
// LDS lookup, then does this step's remaining work (its entries into the stage, the counters)
// while that lookup is in flight.
// row `i` (mod `rows`) of a lane column's LDS array (rows x DEC words): with DEC a power of two the
// array is aligned to its size and the address is one v_and_or_b32, otherwise a v_mad_u32_u24
#define RJ_HL_COLW(i, rows, mask, base) \
  (kPow2 ? ((((i) << kColShift) & (mask)) | (base)) : (__umul24((i) & ((rows) - 1u), DEC * 4u) + (base)))
__host__ __device__ constexpr uint32_t hl_align(uint32_t bytes) { return (bytes & (bytes - 1)) == 0 ? bytes : 16u; }
#define RJ_HL_STEP(SAFE, SYNC)                                                                                  \
  do {                                                                                                    \
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(e >= RJ_HL_ESC) != 0, 0)) {                          \
      RJ_HL_COUNT_ESC;                                                                                    \
      if (e >= RJ_HL_ESC) e = hl_escape(e, peek, tsh != 21u, acb - lut_a, s_lut, tset, pat >> b);         \
      asm volatile("" : "+v"(e)); /* settled here: the join needs no wait for the LDS writes */          \
    }                                                                                                     \
    /* ---- the chain: bit position, block / table state, the next lookup ---- */                      \
    const uint32_t qold = q;                                                                              \
    const uint32_t R1 = (e >> 25) & 63u, n1 = (e >> 16) & 31u;                                            \
    const uint32_t k1 = k + R1 + 1u;                                                                      \
    /* the second symbol: present, and the first leaves the block open */                            \
    bool use2 = (e & RJ_HL_PAIR) != 0u && k1 < 64u;                                                       \
    if (SAFE) use2 = use2 && !skip;                                                                       \
    const uint32_t n2 = e & 31u, R2 = (e >> 9) & 63u;                                                     \
    q -= n1 + (use2 ? n2 : 0u);                                                                           \
    uint32_t kn = use2 ? k1 + R2 + 1u : k1;                                                               \
    if (SAFE) kn = skip ? 64u : kn;                                                                       \
    {                                                                                                     \
      const bool adv = (qold ^ q) > 31u; /* the bit position entered the next word */                   \
      wa = adv ? wb : wa;                                                                                 \
      wb = adv ? wc : wb;                                                                                 \
      rr += adv ? 1u : 0u;                                                                                \
    }                                                                                                     \
    const bool bend = kn >= 64u;                                                                          \
    const uint32_t kcur = k;                                                                              \
    k = bend ? 0u : kn;                                                                                   \
    const uint32_t bn = b + 2u == nb2 ? 0u : b + 2u;                                                      \
    b = bend ? bn : b;                                                                                    \
    /* next symbol's table: the new block's DC table, or the current block's AC table */                 \
    /* (table bases are LDS byte addresses: a lookup is one shift and one shift-add) */                 \
    acb = bend ? __umul24(__builtin_amdgcn_ubfe(pat_ac, b, 1u), uint32_t(RJ_HL_AC_BYTES)) + lut_a : acb;  \
    const uint32_t dcb = (__builtin_amdgcn_ubfe(pat, b, 1u) << (RJ_HL_DC_BITS + 2)) + lut_dc;              \
    const uint32_t tbn = bend ? dcb : acb;                                                                \
    const uint32_t tshn = bend ? uint32_t(32 - RJ_HL_DC_BITS) : uint32_t(32 - RJ_HL_AC_BITS);            \
    const uint32_t peekn = __builtin_amdgcn_alignbit(wa, wb, q);                                          \
    const uint32_t en = lds_rd(((peekn >> tshn) << 2) + tbn);                                             \
    wc = lds_rd(RJ_HL_COLW(rr, RJ_HL_WORDS, kRingMask, ring_a));                                                  \
    /* ---- this step's entries, while the lookup is in flight ---- */                                  \
    /* a coefficient: HUFF_EXTEND of the s extra bits (the low s of the symbol's n bits,            \
       right-aligned), and its position clamped to 63 (libjpeg's natural-order table) */            \
    const uint32_t s1 = (e >> 21) & 15u;                                                                  \
    const uint32_t xb = __builtin_amdgcn_ubfe(peek, 32u - n1, s1); /* the low s of the top n bits */    \
    const uint32_t xm = __builtin_amdgcn_ubfe(0xFFFFFFFFu, 0u, s1);                                       \
    const uint32_t xv = xb > xm - xb ? xb : xb - xm; /* top extra bit clear: negative */               \
    const uint32_t xp = min(kcur + R1, 63u);                                                              \
    uint32_t entry = __builtin_amdgcn_perm(xp, xv, 0x05040100u); /* value's low half | position << 16 */ \
    uint32_t emit = (kcur == 0u || s1 != 0u) ? 1u : 0u; /* DC always; AC coefficients */              \
    if (SAFE) {                                                                                           \
      entry = skip ? RJ_RE_ZERO : entry; /* libjpeg: the rest of the interval is zero blocks */          \
      emit = skip ? 1u : emit;                                                                            \
      emit = blocks_left > 0 ? emit : 0u;                                                                 \
    }                                                                                                     \
    lds_wr(RJ_HL_COLW(ne, kStage, kStageMask, stage_a), entry); /* a non-emitted write: the next free slot */ \
    ne += emit;                                                                                           \
    {                                                                                                     \
      const uint32_t s2 = (e >> 5) & 15u;                                                                 \
      const uint32_t xb2 = __builtin_amdgcn_ubfe(peek, 32u - n1 - n2, s2);                                \
      const uint32_t xm2 = __builtin_amdgcn_ubfe(0xFFFFFFFFu, 0u, s2);                                    \
      const uint32_t xv2 = xb2 > xm2 - xb2 ? xb2 : xb2 - xm2;                                             \
      const uint32_t xp2 = min(k1 + R2, 63u);                                                             \
      uint32_t emit2 = (use2 && s2 != 0u) ? 1u : 0u;                                                      \
      if (SAFE) emit2 = blocks_left > 0 ? emit2 : 0u;                                                     \
      lds_wr(RJ_HL_COLW(ne, kStage, kStageMask, stage_a), __builtin_amdgcn_perm(xp2, xv2, 0x05040100u));   \
      ne += emit2;                                                                                        \
    }                                                                                                     \
    if (SAFE) {                                                                                           \
      const bool act = blocks_left > 0;                                                                   \
      blocks_left -= (bend && act) ? 1u : 0u;                                                             \
      skip = skip || (bend && bn == 0u && (0u - q) > nbits);                                              \
      if (kSplit) { /* a tail stops at libjpeg's insufficient-data point (K2 zero-fills a short tail) */ \
        tdone = (skip && tail && blocks_left != 0u) ? blocks - blocks_left : tdone;                         \
        blocks_left = (skip && tail) ? 0u : blocks_left;                                                    \
      }                                                                                                   \
    } else {                                                                                              \
      blocks_left -= bend ? 1u : 0u;                                                                      \
    }                                                                                                     \
    if (SYNC) {                                                                                           \
      const bool ms = bend && bn == 0u; /* the next symbol starts an MCU */                              \
      mpos = ms ? (0u - q) : mpos;                                                                        \
      mleft = ms ? blocks_left : mleft;                                                                   \
      mseen = mseen || ms;                                                                                \
      recs[min(nr, kRec) * kPairs] = uint16_t(0u - q);                                                     \
      if (kRecNe) rnes[min(nr, kRec) * kPairs] = uint16_t(ne); /* the tail's entries before that MCU */   \
      nr += (ms && nr < kRec) ? 1u : 0u;                                                                  \
    }                                                                                                     \
    e = en;                                                                                               \
    peek = peekn;                                                                                         \
    tsh = tshn;                                                                                           \
  } while (0)

// LDS lane columns shared by a decoder lane and its mover lane: plain LDS words whose order of
// execution is the program order of each wave (the LDS pipeline serves a wave's requests in
// order), read / written as volatile so that the compiler keeps that order too.
// (explicitly in the LDS address space: a volatile generic pointer becomes a system-coherent
// flat access, which waits for every outstanding store of the wave)
typedef __attribute__((address_space(3))) volatile uint32_t lds_vu32;
__device__ __forceinline__ uint32_t lds_ld(const uint32_t *p) { return *(const lds_vu32 *)(p); }
__device__ __forceinline__ void lds_st(uint32_t *p, uint32_t v) { *(lds_vu32 *)(p) = v; }
// plain LDS words by byte address (RJ_HL_STEP: the address arithmetic stays two VALU operations)
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)(p);
}
__device__ __forceinline__ uint32_t lds_rd(uint32_t a) { return *(const lds_u32 *)(uintptr_t)(a); }
__device__ __forceinline__ void lds_wr(uint32_t a, uint32_t v) { *(lds_u32 *)(uintptr_t)(a) = v; }
#define RJ_HL_FIN 0xFFFFFFFFu  // decoder -> mover: the lane's decode is over

// Live rows (rj_device.h RjLive): the active lanes of one decoder wave whose `pub` is set have
// finished their intervals (entries flushed, pieces written); publish their MCU rows.  The
// release is the guide's valid producer form (MI355X_MICROARCH.md, inter-workgroup visibility):
// this wave's stores drained, agent-scope release (the XCD's L2 written back), drained again,
// then one 8-B sc1 store per row -- data and tag in one granule, polled by the consumer.
__device__ __forceinline__ void hl_publish(const RjLive &lv, bool pub, uint32_t img, uint32_t row) {
  const uint64_t m = __builtin_amdgcn_ballot_w64(pub);
  if (m == 0) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifndef RJ_EXP_LIVE_NOFENCE  // timing build: the release's cost (rows may then be read stale)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  const uint32_t lane = __lane_id(), leader = uint32_t(__builtin_ctzll(m));
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(&lv.ctr[RJ_LIVE_RESERVED], uint32_t(__builtin_popcountll(m)));
  base = __shfl(base, int(leader));
  if (pub) {
    const uint32_t r = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
    const uint64_t v = uint64_t(lv.epoch) | (uint64_t((img << RJ_LIVE_ROW_BITS) | row) << 32);
    __hip_atomic_store(&lv.slot[base + r], (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Workgroup = DEC decoder lanes + one mover wave per decoder wave.  Lane `g` of
// [lane0, lane0 + nlanes): the interval rj_lane_seg(g), decoded by decoder lane g % DEC; mover
// lane g % DEC + DEC keeps that lane's bit ring filled.  The decoder never waits on vector
// memory: its only VMEM operations are the entry flushes (fire and forget), so no store latency
// couples into its symbol chain (vmcnt counts loads and stores in one queue -- a decoder that also
// issued its ring loads waited for its older stores).
//
// kSplit (the outlier intervals of a call; two workgroups per CU): an interval listed with
// RJ_LANE_HEAD at lane l < 32 of a wave also has a tail lane at l + 32 (RJ_LANE_TAIL), which
// decodes speculatively from the split byte rj_split_byte(dst_len) as if an MCU started there,
// recording the bit positions of its first RJ_HL_REC MCU starts past the split.  The
// head decodes from the interval start; past the split it compares each MCU start with the
// tail's records.  Huffman codes resynchronise: at the first equal MCU start both decoders are in
// the same state, so the head stops there and the interval becomes two pieces -- the head's
// blocks before that MCU, and the tail's blocks after its first (record + 1) MCUs: the tail notes
// its entry count with each record, so its piece starts at that entry and K2 walks no skipped
// blocks (lean raw entries carry DC differences, so no DC correction is needed).  With no equal MCU start the head decodes the whole interval.  A tail that reaches libjpeg's insufficient-data point stops: K2 zero-fills
// the piece's missing blocks exactly as libjpeg's zero blocks.
template <int DEC, int GROUP, bool kSplit, int PHASE>
__global__ __launch_bounds__(2 * DEC, 2) void k_huff(
    const RjImageDev *__restrict__ imgs, int nimg, uint32_t lane0, uint32_t nlanes, const uint8_t *__restrict__ destuffed,
    const RjTableSet *__restrict__ tabsets, const RjLeanTables *__restrict__ lean, RjCoefBuf coefs, RjHuffSplit split,
    RjLive live) {
  constexpr uint32_t kStage = 2 * GROUP;
  constexpr bool kPow2 = (DEC & (DEC - 1)) == 0;
  constexpr uint32_t kColShift = kPow2 ? __builtin_ctz(DEC * 4u) : 0u;  // bytes between a lane column's words
  // the stage and the ring are aligned to their own size: a word's LDS address is its lane
  // column's address OR its row bits (one v_and_or_b32)
  constexpr uint32_t kStageMask = (kStage << kColShift) - (1u << kColShift);
  constexpr uint32_t kRingMask = (RJ_HL_WORDS << kColShift) - (1u << kColShift);
  static_assert(DEC % 64 == 0, "whole decoder waves");
  // a phase adds <= 2 PHASE entries to < GROUP pending ones: the stage must hold them
  static_assert(2 * PHASE <= GROUP + 1, "stage too small for a phase of two-symbol steps");
  constexpr uint32_t kPairs = kSplit ? DEC / 2 : 1;
  __shared__ __attribute__((aligned(hl_align(RJ_HL_WORDS * DEC * 4)))) uint32_t s_ring[RJ_HL_WORDS][DEC];
  __shared__ __attribute__((aligned(hl_align(kStage * DEC * 4)))) uint32_t s_stage[kStage][DEC];
  __shared__ __attribute__((aligned(16))) uint32_t s_lut[RJ_HL_LUT_WORDS];
  __shared__ uint32_t s_dec[DEC];  // decoder -> mover: ring words fully consumed (RJ_HL_FIN: done)
  __shared__ uint32_t s_mov[DEC];  // mover -> decoder: 16-B chunks committed to the ring
  constexpr uint32_t kRec = RJ_HL_REC;  // MCU-start records per tail lane
  // the tail's entry count with each record, so its piece starts past the skipped MCUs (not in
  // the two-workgroups-per-CU instance: two workgroups must fit in LDS; its tail pieces carry the
  // skip, which K2 walks)
  constexpr bool kRecNe = kSplit && GROUP >= RJ_HL_GROUP;
  __shared__ uint16_t s_rec[kSplit ? kRec + 1 : 1][kPairs];  // tail lanes' MCU-start records (+ scratch)
  __shared__ uint16_t s_rne[kRecNe ? kRec + 1 : 1][kRecNe ? kPairs : 1];  // ... and the tail's entry count at each
  __shared__ uint32_t s_nrec[kPairs];  // records published by the tail (bit 31: no more will come)
  __shared__ uint32_t s_tdone[kPairs];  // blocks a tail decoded before it stopped (0xFFFFFFFF: never stopped)
  __shared__ uint32_t s_T, s_ne;
  const uint32_t tid = threadIdx.x;
  const bool mover = tid >= uint32_t(DEC);
  const uint32_t L = mover ? tid - DEC : tid;  // the decoder lane (LDS column)
  if (tid == 0) s_ne = 0;
  if (live.slot != nullptr && tid == 0) {  // this CU runs K1 (live K2 waits there until it is done)
    atomicAdd(&live.cu_busy[rj_live_cu_key()], 1u);
    atomicAdd(&live.ctr[RJ_LIVE_STARTED], 1u);
  }
  const uint32_t g = lane0 + blockIdx.x * DEC + L;
  bool pending = g < lane0 + nlanes;
  uint32_t gseg = 0, role = 0;
  if (pending) {
    const uint32_t e = rj_lane_seg(coefs, g);
    pending = e != 0xFFFFFFFFu;
    gseg = kSplit ? e & ~(RJ_LANE_HEAD | RJ_LANE_TAIL) : e;
    role = kSplit ? e & (RJ_LANE_HEAD | RJ_LANE_TAIL) : 0u;
  }
  const bool head = kSplit && role == RJ_LANE_HEAD;
  const bool tail = kSplit && role == RJ_LANE_TAIL;
  const uint32_t pair = (L >> 6) * 32u + (L & 31u);  // a head lane and its tail share the record column
  int i = 0;
  if (pending) i = upper_index(nimg, gseg, [&](int qq) { return imgs[qq].seg_prefix; });
  const RjImageDev &im = imgs[i];
  const uint32_t my_ts = im.tabset;
  // one pass per distinct table set among the workgroup's lanes (normally exactly one)
  while (__syncthreads_or(pending)) {
    if (tid == 0) s_T = 0xFFFFFFFFu;
    __syncthreads();
    if (pending) atomicMin(&s_T, my_ts);
    if (!mover) {
      s_dec[L] = 0;
      s_mov[L] = 0;
    }
    __syncthreads();
    const uint32_t T = s_T;
    {
      const uint4 *src = reinterpret_cast<const uint4 *>(lean + T);
      uint4 *d4 = reinterpret_cast<uint4 *>(s_lut);
      for (uint32_t w = tid; w < RJ_HL_LUT_WORDS / 4; w += 2 * DEC) d4[w] = gp(src)[w];
    }
    __syncthreads();
    if (!(pending && my_ts == T)) continue;
    pending = false;
    const uint32_t seg = gseg - im.seg_prefix;
    const RjSegDev sg = gp(im.segs)[seg];
    // split intervals: the tail's bytes start at the split byte
    const uint32_t sp_byte = (head || tail) ? rj_split_byte(sg.dst_len) : 0u;
    const uint32_t nbytes = tail ? sg.dst_len - sp_byte : sg.dst_len;
    const uint4 *src = reinterpret_cast<const uint4 *>(destuffed + im.destuff_off + sg.dst_off + (tail ? sp_byte : 0u));
    const uint32_t nchunks = (nbytes + 15) / 16;
    const HCol<DEC> ring{&s_ring[0][L]};

    if (mover) {
      // ---- mover: keep the ring's free chunk slots filled (past the data: zero chunks, the
      // zero bits libjpeg inserts), up to 4 chunks per round; a round's loads are committed at
      // the start of the next round, so each round waits for loads issued one round earlier ----
      uint32_t cm = 0, na = 0;
      uint4 p0 = make_uint4(0, 0, 0, 0), p1 = p0, p2 = p0, p3 = p0;
      for (;;) {
        const uint32_t rd = lds_ld(&s_dec[L]);
        if (na > 0) {
          hl_put(ring, cm & (RJ_HL_CHUNKS - 1), p0);
          if (na > 1) hl_put(ring, (cm + 1) & (RJ_HL_CHUNKS - 1), p1);
          if (na > 2) hl_put(ring, (cm + 2) & (RJ_HL_CHUNKS - 1), p2);
          if (na > 3) hl_put(ring, (cm + 3) & (RJ_HL_CHUNKS - 1), p3);
          cm += na;
          lds_st(&s_mov[L], cm);  // after the ring words (same wave, in order)
          na = 0;
        }
        const bool fin = rd == RJ_HL_FIN;
        // chunk slots below the decoder's oldest live word are free
        const uint32_t live = fin ? RJ_HL_CHUNKS : cm - (rd >> 2);
        const uint32_t n = min(RJ_HL_CHUNKS - live, 4u);
        if (n > 0) {
          p0 = *gp(cm < nchunks ? src + cm : rj_hl_zero);
          if (n > 1) p1 = *gp(cm + 1 < nchunks ? src + cm + 1 : rj_hl_zero);
          if (n > 2) p2 = *gp(cm + 2 < nchunks ? src + cm + 2 : rj_hl_zero);
          if (n > 3) p3 = *gp(cm + 3 < nchunks ? src + cm + 3 : rj_hl_zero);
          na = n;
        }
        if (__builtin_amdgcn_ballot_w64(!fin) == 0) break;
        if (__builtin_amdgcn_ballot_w64(n > 0) == 0) __builtin_amdgcn_s_sleep(4);
      }
      continue;
    }

    // ---- decoder ----
    const uint32_t nblk = im.nblk_mcu;
    uint32_t pat = 0;  // per block b: bit 2b its DC table, bit 2b + 1 its AC table
    for (uint32_t bb = 0; bb < nblk; bb++) {
      const uint32_t cc = im.blk_comp[bb] & 3;
      pat |= ((im.comp_td[cc] & 1u) | ((im.comp_ta[cc] & 1u) << 1)) << (2 * bb);
    }
    const uint32_t nb2 = 2 * nblk;
    const uint32_t pat_ac = pat >> 1;  // bit 2b: block b's AC table
    const uint32_t nbits = nbytes * 8u;
    const uint32_t blocks = sg.mcu_count * nblk;
    // entry regions: the interval's own; a tail lane writes its pair's slot of the split region
    const uint64_t tail_abs = kSplit ? split.ent + uint64_t((g >> 6) * 32u + (g & 31u)) * split.cap : 0u;
    const uint64_t ent_abs = tail ? tail_abs : im.ent_off + sg.ent_off;
    uint32_t *ent = coefs.ent + ent_abs;
#ifdef RJ_EXP_E16
#define RJ_HL_DST(f) reinterpret_cast<uint32_t *>(reinterpret_cast<uint16_t *>(coefs.ent) + ent_abs + (f))
#else
#define RJ_HL_DST(f) (ent + (f))
#endif
    RjPiece *piece = coefs.piece + rj_seg_lane0_k<kSplit>(coefs, gseg);
    const RjTableSet *tset = tabsets + T;  // canonical search (escape path)
    const HCol<DEC> stage{&s_stage[0][L]};
    const uint32_t stage_a = lds_addr(&s_stage[0][L]), ring_a = lds_addr(&s_ring[0][L]);
    const uint32_t lut_a = lds_addr(s_lut), lut_dc = lut_a + RJ_HL_DC0;
    // split state: records (tail), the last MCU start seen (head), the head's scan over the records
    uint16_t *const recs = &s_rec[0][kSplit ? pair : 0u];
    uint16_t *const rnes = &s_rne[0][kRecNe ? pair : 0u];
    uint32_t nr = tail ? 0u : kRec;
    uint32_t mpos = 0, mleft = 0, jrec = 0, blk_head = 0, ne_tail = 0, skip_tail = 0, tdone = 0xFFFFFFFFu;
    bool mseen = false, synced = false, checking = head;
    const uint32_t sp_bits = sp_byte * 8u;
    if (tail) lds_st(&s_nrec[pair], 0u);
    // a phase reads ring words up to rr + 8 (8 symbols of <= 31 bits, the last one's read-ahead)
// (avail: ring words known to be committed; the decoder re-reads the mover's count only when a
// lane's next phase could read past them)
#define RJ_HL_WAIT_RING(upto)                                                                     \
  {                                                                                               \
    uint32_t cmv = lds_ld(&s_mov[L]);                                                             \
    while (__builtin_amdgcn_ballot_w64(4u * cmv < (upto)) != 0) {                                 \
      __builtin_amdgcn_s_sleep(2);                                                                \
      cmv = lds_ld(&s_mov[L]);                                                                    \
    }                                                                                             \
    avail = 4u * cmv;                                                                             \
    asm volatile("" ::: "memory");                                                                \
  }
    uint32_t avail = 0;
    RJ_HL_WAIT_RING(uint32_t(PHASE) + 2u);  // words 0 .. PHASE + 1 (a phase reads up to rr + PHASE)
    uint32_t q = 0;               // -(bits consumed)
    // q = 0 is bit 0: alignbit(wa, wb, 0) would return wb, so the window starts one word back
    // (words -1, 0; j = (pos - 1) >> 5): wa is a dummy word whose bits are never returned
    uint32_t wa = 0, wb = ring[0], wc = ring[1];
    uint32_t rr = 1;  // ring index of wc
    uint32_t ne = 0, fl = 0;
    bool skip = (sg.flags & RJ_SEG_MISSING) != 0;
    uint32_t blocks_left = blocks;
    uint32_t b = 0, k = 0;
    uint32_t acb = ((pat >> 1) & 1u) * uint32_t(RJ_HL_AC_BYTES) + lut_a;  // LDS byte address
    uint32_t tb = RJ_HL_DC0 + ((pat & 1u) << (RJ_HL_DC_BITS + 2));
    uint32_t tsh = 32 - RJ_HL_DC_BITS;
    // the first symbol's peek and table entry (RJ_HL_STEP is software-pipelined)
    uint32_t peek = __builtin_amdgcn_alignbit(wa, wb, q);
    uint32_t e = s_lut[(tb >> 2) + (peek >> tsh)];
#ifdef RJ_HL_STAMPS
    uint64_t st_steps = 0, st_end = 0, st_fast = 0, st_safe = 0, st_esc = 0, st_flush = 0, st_waits = 0;
    const uint64_t st_begin = __builtin_amdgcn_s_memtime();
    const uint64_t st_begin_rt = __builtin_amdgcn_s_memrealtime();
#define RJ_HL_T0 const uint64_t t0 = __builtin_amdgcn_s_memtime()
#define RJ_HL_T1(fast)                                  \
  const uint64_t t1 = __builtin_amdgcn_s_memtime();     \
  st_steps += t1 - t0;                                  \
  if (fast) st_fast++;                                  \
  else st_safe++
#define RJ_HL_T2 st_end += __builtin_amdgcn_s_memtime() - t1
#define RJ_HL_TF st_flush += __builtin_amdgcn_s_memtime() - t1
#define RJ_HL_TW st_waits++
#else
#define RJ_HL_TF
#define RJ_HL_TW
#define RJ_HL_T0
#define RJ_HL_T1(fast)
#define RJ_HL_T2
#endif
    while (__builtin_amdgcn_ballot_w64(blocks_left > 0) != 0) {
      if (blocks_left == 0) continue;  // finished lanes sit out the rest of the wave's phases
      RJ_HL_T0;
      // no live lane can finish its blocks or reach its data's end in this phase: the lean body
      const bool safe = __builtin_amdgcn_ballot_w64(
                            !(blocks_left >= PHASE && !skip && (0u - q) + PHASE * 31u < nbits)) != 0;
      // split: a tail still recording, or a head that may pass an MCU start beyond the split
      const bool sync = kSplit && __builtin_amdgcn_ballot_w64(
                                      nr < kRec || (checking && (0u - q) + PHASE * 31u >= sp_bits)) != 0;
      if (!safe && !sync) {
#pragma unroll
        for (uint32_t s_ = 0; s_ < PHASE; s_++) RJ_HL_STEP(false, false);
      } else if (!safe) {
#pragma unroll
        for (uint32_t s_ = 0; s_ < PHASE; s_++) RJ_HL_STEP(false, kSplit);
      } else {
#pragma unroll
        for (uint32_t s_ = 0; s_ < PHASE; s_++) RJ_HL_STEP(true, kSplit);
      }
      RJ_HL_T1(!safe);
      // ---- phase end: words below rr - 2 (the one in wa) are free for the mover; a full stage
      // group leaves (< GROUP stay pending); wait until the next phase's words are in the ring ----
      // (rr = 1 until the first word is used up: rr - 2 would read as RJ_HL_FIN)
      lds_st(&s_dec[L], max(rr, 2u) - 2u);
      if (ne - fl >= GROUP) {
        hl_flush<DEC, GROUP>(stage, fl, RJ_HL_DST(fl));
        fl += GROUP;
      }
      RJ_HL_TF;
      if (kSplit) {
        if (tail) {  // publish the records (16-bit positions: the next phase must stay below 2^16)
          if ((0u - q) >= RJ_HL_REC_LIMIT) nr = kRec;
          lds_st(&s_nrec[pair], nr | ((nr >= kRec || blocks_left == 0) ? 0x80000000u : 0u));
        }
        if (checking && mseen && mpos >= sp_bits) {
          // head: is its last MCU start one of the tail's?  (records are in position order)
          const uint32_t rel = mpos - sp_bits;
          const uint32_t pub = lds_ld(&s_nrec[pair]);
          const uint32_t nrec = pub & 0xFFFFu;
          uint32_t r = 0;
          while (jrec < nrec) {
            r = *(const __attribute__((address_space(3))) volatile uint16_t *)(&recs[jrec * kPairs]);
            if (r >= rel) break;
            jrec++;
          }
          if (jrec < nrec && r == rel) {
            synced = true;  // same state from here on: the rest is the tail's
            checking = false;
            blk_head = blocks - mleft;
            // record j: after the tail's first j + 1 MCUs, whose entries the tail piece starts past
            if (kRecNe) ne_tail = *(const __attribute__((address_space(3))) volatile uint16_t *)(&rnes[jrec * kPairs]);
            else skip_tail = (jrec + 1) * nblk;
            blocks_left = 0;
          } else if (jrec >= nrec && (pub >> 31) != 0) {
            checking = false;  // no record left to meet: the head decodes the whole interval
          }
        }
        mseen = false;
      }
#ifdef RJ_HL_EAGER_RING
      if (true) {
#else
      if (__builtin_amdgcn_ballot_w64(avail < rr + PHASE + 1u) != 0) {
#endif
        RJ_HL_TW;
        RJ_HL_WAIT_RING(rr + PHASE + 1u);
        wc = ring[rr & (RJ_HL_WORDS - 1)];  // the last step's read-ahead may predate the commit
      }
      RJ_HL_T2;
    }
    lds_st(&s_dec[L], RJ_HL_FIN);
    if (kSplit && tail) lds_st(&s_tdone[pair], tdone);  // before its head (same wave) writes the pieces
#ifdef RJ_HL_STAMPS
    if ((tid & 63) == 0) {
      atomicAdd(&rj_hl_stamp[0], (unsigned long long)st_steps);
      atomicAdd(&rj_hl_stamp[1], (unsigned long long)st_end);
      atomicAdd(&rj_hl_stamp[2], (unsigned long long)st_fast);
      atomicAdd(&rj_hl_stamp[3], (unsigned long long)st_safe);
      atomicAdd(&rj_hl_stamp[4], 1ull);
      atomicAdd(&rj_hl_stamp[5], (unsigned long long)st_esc);
      const unsigned long long st_loop = __builtin_amdgcn_s_memtime() - st_begin;
      atomicAdd(&rj_hl_stamp[6], st_loop);
      atomicMax(&rj_hl_stamp[7], st_loop);
      atomicAdd(&rj_hl_stamp[8], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - st_begin_rt));
      atomicAdd(&rj_hl_stamp[9], (unsigned long long)st_flush);
      atomicAdd(&rj_hl_stamp[10], (unsigned long long)st_waits);
    }
#endif
    stage[ne & (kStage - 1)] = RJ_RE_TERM;
    while (fl < ne + 1) {  // [fl, ne]: at most 2 GROUP entries, the terminator included
      hl_flush<DEC, GROUP>(stage, fl, RJ_HL_DST(fl));
      fl += GROUP;
    }
    if (!tail) {
      if (synced) {
        gp(piece)[0] = RjPiece{ent_abs, 0u, blk_head, 2u, {0, 0, 0}};
        // the tail piece's npieces: the blocks K2 passes over first (0 when the piece starts at
        // the recorded entry), bit 31 when the tail stopped short of its blocks (K2 then checks
        // for its terminator and zero-fills the rest)
        const uint32_t need = (jrec + 1) * nblk + (blocks - blk_head);
        const uint32_t early = lds_ld(&s_tdone[pair]) < need ? 0x80000000u : 0u;
        gp(piece)[1] = RjPiece{tail_abs + ne_tail, blk_head, blocks - blk_head, skip_tail | early, {0, 0, 0}};
      } else {
        *gp(piece) = RjPiece{ent_abs, 0u, blocks, 1u, {0, 0, 0}};
      }
    }
    // live rows: a whole interval's row (or a split head's that met no tail record) is complete;
    // a synced split row is two pieces, left to the split-aware K2 instance
    if (live.slot != nullptr) hl_publish(live, !tail && !synced, uint32_t(i), seg);
    if (coefs.count) atomicAdd(&s_ne, ne + 1);
  }
  // (every wave left the loop at its last barrier: the workgroup's decoding is over)
  if (live.slot != nullptr && tid == 0) atomicSub(&live.cu_busy[rj_live_cu_key()], 1u);
  if (live.slot != nullptr && !mover && (tid & 63u) == 0) {  // this decoder wave is done (after its rows)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t d = __hip_atomic_fetch_add(&live.ctr[RJ_LIVE_DONE], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    if (d + 1u == live.k1_waves) {  // the last one: close the tickets; k_rows_rest takes what is left
      const uint32_t t = atomicOr(&live.ctr[RJ_LIVE_TICKET], RJ_LIVE_CLOSED);
      __hip_atomic_store(&live.ctr[RJ_LIVE_FINAL], t & ~RJ_LIVE_CLOSED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (tid == 0 && coefs.count != nullptr && s_ne != 0) atomicAdd(coefs.count, (unsigned long long)s_ne);
}

// ---------------------------------------------------------------------------------------
// Chunk lanes (k_huff_chunk): K1 of calls whose intervals are not all MCU rows -- long or
// restart-less intervals (every reference fixture, BASELINE's C2 no-DRI
// twin; small calls, whose intervals the call cuts to fill the chip).  The lean machinery above
// (mover waves, one table entry per code with its follower, the software-pipelined step) over
// the chunk layout of rj_entropy.hip: an interval of rj_nch > 1 chunks gets one lane per chunk
// (reverse order, regions at RjCoefBuf.seg_ent), chunk c > 0 starts
// speculatively at its first byte as if a Y block began there and records its state every
// RJ_RECORD_EVERY block starts; a lane that runs past its own end compares its block starts with
// the records of the chunk it entered and stops at the first equal state.  Records, the per-lane
// result (RjChunkRes), k_resolve and the serial fallback (k_entropy<true>) are rj_entropy.hip's,
// unchanged.  Entries carry ABSOLUTE DC values (the lane keeps libjpeg's three predictors; a
// speculative chunk's are corrected per piece by k_resolve), so the images of such a call take
// K2's DC-correcting path (dc_diff = 0).  Intervals of one chunk are decoded whole, exactly
// (libjpeg's insufficient-data and missing-marker rules, as the lean launch), into one piece.
template <int kScope>
__device__ __forceinline__ void hc_put_record(RjRecord *r, uint32_t pos, uint32_t b, uint32_t epoch, uint32_t ne,
                                              uint32_t rb, int p0, int p1, int p2) {
  *gp(reinterpret_cast<int4 *>(&r->pred[0])) = make_int4(p0, p1, p2, 0);
  if (kScope == __HIP_MEMORY_SCOPE_WORKGROUP) {
    *gp(reinterpret_cast<uint4 *>(r)) = make_uint4(pos, (b & 15u) | (epoch << 4), ne, rb);
  } else {
    *gp(reinterpret_cast<uint2 *>(&r->ne)) = make_uint2(ne, rb);
    __hip_atomic_store(reinterpret_cast<uint64_t *>(r), uint64_t(pos) | (uint64_t((b & 15u) | (epoch << 4)) << 32),
                       __ATOMIC_RELAXED, kScope);
  }
}

// The chunk-lane step: RJ_HL_STEP plus the DC predictors (absolute DC entries) and, at a block
// end of a chunk lane, its records / sync search / stop conditions (SAFE phases only: a lane
// inside its own chunk cannot stop).
#define RJ_HC_STEP(SAFE)                                                                                        \
  do {                                                                                                    \
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(e >= RJ_HL_ESC) != 0, 0)) {                          \
      if (e >= RJ_HL_ESC) e = hl_escape(e, peek, tsh != 21u, acb - lut_a, s_lut, tset, pat >> b);         \
      asm volatile("" : "+v"(e)); /* settled here: the join needs no wait for the LDS writes */          \
    }                                                                                                     \
    const uint32_t qold = q;                                                                              \
    const uint32_t R1 = (e >> 25) & 63u, n1 = (e >> 16) & 31u;                                            \
    const uint32_t k1 = k + R1 + 1u;                                                                      \
    bool use2 = (e & RJ_HL_PAIR) != 0u && k1 < 64u;                                                       \
    if (SAFE) use2 = use2 && !skip;                                                                       \
    const uint32_t n2 = e & 31u, R2 = (e >> 9) & 63u;                                                     \
    q -= n1 + (use2 ? n2 : 0u);                                                                           \
    uint32_t kn = use2 ? k1 + R2 + 1u : k1;                                                               \
    if (SAFE) kn = skip ? 64u : kn;                                                                       \
    {                                                                                                     \
      const bool adv = (qold ^ q) > 31u;                                                                  \
      wa = adv ? wb : wa;                                                                                 \
      wb = adv ? wc : wb;                                                                                 \
      rr += adv ? 1u : 0u;                                                                                \
    }                                                                                                     \
    const bool bend = kn >= 64u;                                                                          \
    const uint32_t kcur = k, bcur = b;                                                                    \
    k = bend ? 0u : kn;                                                                                   \
    const uint32_t bn = b + 2u == nb2 ? 0u : b + 2u;                                                      \
    b = bend ? bn : b;                                                                                    \
    /* (table bases are LDS byte addresses: a lookup is one shift and one shift-add) */                 \
    acb = bend ? __umul24(__builtin_amdgcn_ubfe(pat_ac, b, 1u), uint32_t(RJ_HL_AC_BYTES)) + lut_a : acb;  \
    const uint32_t dcb = (__builtin_amdgcn_ubfe(pat, b, 1u) << (RJ_HL_DC_BITS + 2)) + lut_dc;              \
    const uint32_t tbn = bend ? dcb : acb;                                                                \
    const uint32_t tshn = bend ? uint32_t(32 - RJ_HL_DC_BITS) : uint32_t(32 - RJ_HL_AC_BITS);            \
    const uint32_t peekn = __builtin_amdgcn_alignbit(wa, wb, q);                                          \
    const uint32_t en = lds_rd(((peekn >> tshn) << 2) + tbn);                                             \
    wc = lds_rd(((rr << kColShift) & kRingMask) | ring_a);                                                  \
    /* ---- entries; a DC symbol's value is the predictor of its block's component + the difference */ \
    const uint32_t s1 = (e >> 21) & 15u;                                                                  \
    const uint32_t xb = __builtin_amdgcn_ubfe(peek, 32u - n1, s1);                                        \
    const uint32_t xm = __builtin_amdgcn_ubfe(0xFFFFFFFFu, 0u, s1);                                       \
    const uint32_t xv = xb > xm - xb ? xb : xb - xm;                                                      \
    const bool isdc = kcur == 0u;                                                                         \
    const uint32_t cc = (cpat >> bcur) & 3u;                                                              \
    const int pdc = (cc == 0u ? pred0 : (cc == 1u ? pred1 : pred2)) + int(xv);                            \
    const uint32_t xp = min(kcur + R1, 63u);                                                              \
    uint32_t entry = __builtin_amdgcn_perm(xp, isdc ? uint32_t(pdc) : xv, 0x05040100u);                   \
    uint32_t emit = (isdc || s1 != 0u) ? 1u : 0u;                                                         \
    const bool act = blocks_left > 0;                                                                     \
    if (SAFE) {                                                                                           \
      entry = skip ? 0u : entry; /* libjpeg: the rest of the interval is zero blocks (DC 0, absolute) */  \
      emit = skip ? 1u : emit;                                                                            \
      emit = act ? emit : 0u;                                                                             \
    }                                                                                                     \
    {   /* a stopped lane's predictors stay those of its stop point (RjChunkRes.pred) */                  \
      const bool upd = isdc && (!(SAFE) || (act && !skip));                                               \
      pred0 = (upd && cc == 0u) ? pdc : pred0;                                                            \
      pred1 = (upd && cc == 1u) ? pdc : pred1;                                                            \
      pred2 = (upd && cc == 2u) ? pdc : pred2;                                                            \
    }                                                                                                     \
    lds_wr(((ne << kColShift) & kStageMask) | stage_a, entry);                                          \
    ne += emit;                                                                                           \
    {                                                                                                     \
      const uint32_t s2 = (e >> 5) & 15u;                                                                 \
      const uint32_t xb2 = __builtin_amdgcn_ubfe(peek, 32u - n1 - n2, s2);                                \
      const uint32_t xm2 = __builtin_amdgcn_ubfe(0xFFFFFFFFu, 0u, s2);                                    \
      const uint32_t xv2 = xb2 > xm2 - xb2 ? xb2 : xb2 - xm2;                                             \
      const uint32_t xp2 = min(k1 + R2, 63u);                                                             \
      uint32_t emit2 = (use2 && s2 != 0u) ? 1u : 0u;                                                      \
      if (SAFE) emit2 = act ? emit2 : 0u;                                                                 \
      lds_wr(((ne << kColShift) & kStageMask) | stage_a, __builtin_amdgcn_perm(xp2, xv2, 0x05040100u));   \
      ne += emit2;                                                                                        \
    }                                                                                                     \
    if (SAFE) {                                                                                           \
      blocks_left -= (bend && act) ? 1u : 0u;                                                             \
      skip = skip || (bend && bn == 0u && (0u - q) > nbits_skip);                                         \
    } else {                                                                                              \
      blocks_left -= bend ? 1u : 0u;                                                                      \
    }                                                                                                     \
    if (chunk && bend && act) { /* a block start of a chunk lane (divergent: ~1 step in 6) */           \
      rb++;                                                                                               \
      const uint32_t pos = start_bit + (0u - q);                                                          \
      if (spec && nrec < RJ_MAX_RECORDS && rb >= rec_rb && pos >= own_bit && pos < end_bit && !rp) {        \
        rp = true;                                                                                        \
        rec_rb = rb + RJ_RECORD_EVERY;                                                                    \
        rp_pos = pos;                                                                                     \
        rp_b = b >> 1;                                                                                    \
        rp_ne = ne;                                                                                       \
        rp_rb = rb;                                                                                       \
        rp_p0 = pred0;                                                                                    \
        rp_p1 = pred1;                                                                                    \
        rp_p2 = pred2;                                                                                    \
      }                                                                                                   \
      if (SAFE) {                                                                                         \
        if (pos >= next_tgt_bit && tgt < next_chunks) { /* entered the next later chunk */              \
          tgt++;                                                                                          \
          _Pragma("unroll") for (int hh = 0; hh < NH; hh++) j[hh] = 0;                                     \
          next_tgt_bit += clen_bits;                                                                      \
        }                                                                                                 \
        /* against each phase hypothesis of that chunk (rj_chunk_lanes); lanes still inside their */    \
        /* own chunk (tgt 0) skip the compares */                                                         \
        if (tgt != 0u && status == 0u) {                                                                  \
          _Pragma("unroll") for (int hh = 0; hh < NH; hh++) {                                             \
            if (uint32_t(hh) < H && status == 0 && cache_tj[hh] == (tgt << 16 | j[hh]) &&                  \
                uint32_t(cache[hh] >> 36) == (epoch & 0x0FFFFFFFu)) {                                     \
              const uint32_t cpos = uint32_t(cache[hh]);                                                  \
              if (cpos == pos && uint32_t(cache[hh] >> 32 & 15u) == (b >> 1)) {                           \
                status = RJ_CHUNK_SYNC; /* identical state from here on: the later chunk owns the rest */ \
                s_tgt = tgt | uint32_t(hh) << 16;                                                         \
                s_rec = j[hh];                                                                            \
              } else if (cpos < pos) {                                                                    \
                j[hh]++;                                                                                  \
              }                                                                                           \
            }                                                                                             \
          }                                                                                               \
        }                                                                                                 \
        if (status == 0 && pos >= nbits_abs) {                                                            \
          if (pos > nbits_abs) rb_over = rb - 1;                                                          \
          status = RJ_CHUNK_DONE;                                                                         \
        }                                                                                                 \
        if (status == 0 && (pos > ov_bit || ne + 2 * RJ_ENT_PER_BLOCK > cap)) status = RJ_CHUNK_FAIL;     \
        if (status != 0) blocks_left = 0;                                                                 \
      }                                                                                                   \
    }                                                                                                     \
    e = en;                                                                                               \
    peek = peekn;                                                                                         \
    tsh = tshn;                                                                                           \
  } while (0)

// kHyp chain propagation inside a workgroup (k_huff_chunk): lane X is on its interval's true
// chain; follow the links of the lanes it reaches, marking each on the chain and its chunk decided
// (and the chunks a link jumps over passed by).  Lanes are workgroup-relative; i0 is the interval's
// first lane.  A lane that syncs stores its link, then reads its own mark; the walk sets a mark,
// then reads the link: with sequentially consistent LDS atomics one of the two sees the other, so
// no link is lost (a lane may be walked twice, which only repeats idempotent stores).
template <typename U32>
__device__ __forceinline__ void hc_chain_walk(uint32_t X, uint32_t i0, uint32_t nch, uint32_t H, U32 *s_link, U32 *s_onc,
                                              U32 *s_conf) {
  for (uint32_t guard = 0; guard < 2u * RJ_K1_WG; guard++) {
    const uint32_t T = __hip_atomic_load(&s_link[X], __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (T == 0xFFFFFFFFu) break;
    const uint32_t oT = T - i0, oX = X - i0, c0 = (nch - 1) * H;
    const uint32_t cT = nch - 1 - oT / H, hT = oT - (oT / H) * H;
    const uint32_t cX = oX >= c0 ? 0u : nch - 1 - oX / H;
    for (uint32_t cc = cX + 1; cc < cT; cc++)  // chunks the link jumps over: no hypothesis of theirs is needed
      __hip_atomic_store(&s_conf[i0 + (nch - 1 - cc) * H], 0xFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_store(&s_conf[T - hT], hT + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (__hip_atomic_fetch_or(&s_onc[T], 1u, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_WORKGROUP) != 0) break;
    X = T;
  }
}

// kHyp: the layout with MCU-phase hypotheses (RjCoefBuf.hyp > 1, small calls); the instance
// without keeps one lane per chunk and none of the per-hypothesis state (its registers and
// compares cost a restart-less 1024-image call 8 % of K1 when compiled in).
template <int kScope, bool kHyp>
__global__ __launch_bounds__(512, 1) void k_huff_chunk(const RjImageDev *__restrict__ imgs, int nimg, uint32_t lane0,
                                                      uint32_t nlanes, const uint8_t *__restrict__ destuffed,
                                                      const RjTableSet *__restrict__ tabsets,
                                                      const RjLeanTables *__restrict__ lean, RjCoefBuf coefs,
                                                      uint32_t epoch) {
  constexpr int DEC = RJ_K1_WG;  // the chunk layout's granule (an interval of <= DEC chunks in one workgroup)
  constexpr int GROUP = RJ_HL_GROUP, PHASE = RJ_HL_PHASE;
  constexpr uint32_t kStage = 2 * GROUP;
  constexpr uint32_t kColShift = __builtin_ctz(DEC * 4u);  // bytes between a lane column's words
  // the stage and the ring are aligned to their own size: a word's LDS address is its lane
  // column's address OR its row bits (one v_and_or_b32)
  constexpr uint32_t kStageMask = (kStage << kColShift) - (1u << kColShift);
  constexpr uint32_t kRingMask = (RJ_HL_WORDS << kColShift) - (1u << kColShift);
  static_assert((DEC & (DEC - 1)) == 0, "lane columns: DEC a power of two");
  static_assert(2 * PHASE <= GROUP + 1, "stage too small for a phase of two-symbol steps");
  __shared__ __attribute__((aligned(RJ_HL_WORDS * DEC * 4))) uint32_t s_ring[RJ_HL_WORDS][DEC];
  __shared__ __attribute__((aligned(kStage * DEC * 4))) uint32_t s_stage[kStage][DEC];
  __shared__ __attribute__((aligned(16))) uint32_t s_lut[RJ_HL_LUT_WORDS];
  __shared__ uint32_t s_dec[DEC];
  __shared__ uint32_t s_mov[DEC];
  // kHyp, workgroup-scope layout (an interval's lanes in this workgroup): the chain of pieces as
  // the lanes find it.  s_link[l]: the lane (in the workgroup) lane l synced into; s_onc[l]: lane l
  // is on the interval's true chain (chunk 0's lane from the start, then every lane an on-chain
  // lane synced into); s_conf[first lane of a chunk]: 0 unknown, h + 1 when hypothesis h of that
  // chunk is on the chain, 0xFFFF when the chain passed the chunk by.  A speculative lane past its
  // own end whose chunk is decided for another hypothesis stops: nothing will read its pieces,
  // and a hypothesis that started out of phase may take a long time to fall into step.
  __shared__ uint32_t s_link[kHyp ? DEC : 1], s_onc[kHyp ? DEC : 1], s_conf[kHyp ? DEC : 1];
  __shared__ uint32_t s_T, s_ne;
  const uint32_t tid = threadIdx.x;
  const bool mover = tid >= uint32_t(DEC);
#ifdef RJ_HL_STAMPS
  const uint64_t hc_t_entry = __builtin_amdgcn_s_memtime();
  uint64_t hc_loop = 0, hc_ph = 0, hc_safe = 0, hc_wait = 0, hc_setup = 0, hc_safe_cyc = 0, hc_uns_cyc = 0;
  uint64_t hc_end[4] = {0, 0, 0, 0};  // phase end: s_dec + chain block, record settle, flush; phase start
#endif
  const uint32_t L = mover ? tid - DEC : tid;
  if (tid == 0) s_ne = 0;
  const uint32_t g = lane0 + blockIdx.x * DEC + L;
  bool pending = g < lane0 + nlanes;
  uint32_t gseg = 0, c = 0, h = 0, nch = 1, l_first = 0;
  constexpr int NH = kHyp ? RJ_MAX_HYP : 1;  // hypothesis state slots
  const uint32_t H = kHyp ? coefs.hyp : 1u;
  int i = 0;
  if (pending) {
    gseg = rj_lane_seg(coefs, g);
    pending = gseg != 0xFFFFFFFFu;
  }
  if (pending) {
    i = upper_index(nimg, gseg, [&](int qq) { return imgs[qq].seg_prefix; });
    nch = rj_nch(coefs, gp(imgs[i].segs)[gseg - imgs[i].seg_prefix].src_len);
    // reverse order, later chunks on earlier lanes; each chunk c > 0 under H phase hypotheses
    // (rj_device.h rj_chunk_lane)
    l_first = rj_seg_lane0(coefs, gseg);
    const uint32_t o = g - l_first;
    if (nch > 1 && o < (nch - 1) * H) {
      c = nch - 1 - o / H;
      h = o - (o / H) * H;
    }
  }
  const RjImageDev &im = imgs[i];
  const uint32_t my_ts = im.tabset;
  while (__syncthreads_or(pending)) {
    if (tid == 0) s_T = 0xFFFFFFFFu;
    __syncthreads();
    if (pending) atomicMin(&s_T, my_ts);
    if (!mover) {
      s_dec[L] = 0;
      s_mov[L] = 0;
      if constexpr (kHyp) {
        s_link[L] = 0xFFFFFFFFu;
        s_onc[L] = c == 0 ? 1u : 0u;
        s_conf[L] = 0u;
      }
    }
    __syncthreads();
    const uint32_t T = s_T;
    {
      const uint4 *src = reinterpret_cast<const uint4 *>(lean + T);
      uint4 *d4 = reinterpret_cast<uint4 *>(s_lut);
      for (uint32_t w = tid; w < RJ_HL_LUT_WORDS / 4; w += 2 * DEC) d4[w] = gp(src)[w];
    }
    __syncthreads();
    if (!(pending && my_ts == T)) continue;
    pending = false;
    const uint32_t seg = gseg - im.seg_prefix;
    const RjSegDev sg = gp(im.segs)[seg];
    const bool chunk = nch > 1;
    const uint32_t nbytes = sg.dst_len;
    const uint32_t clen = chunk ? rj_chunk_len(nbytes, nch) : nbytes;
    const uint32_t b0 = chunk ? min(c * clen, nbytes) : 0u, b1 = chunk ? min(b0 + clen, nbytes) : nbytes;
    // no data left for this chunk (16-B rounding), or a phase hypothesis the image's MCU does not have
    const bool empty = chunk && c > 0 && (b0 >= nbytes || h >= uint32_t(im.nblk_mcu));
    // a speculative lane starts `warm` bytes before its chunk, so that its decode has usually
    // resynchronised with the true one by the chunk start, where its records begin: the lane
    // before then meets a record right after it crosses, instead of running on through the
    // (long-tailed) resynchronisation distance itself.  At most half a chunk (the lane has to be
    // past its chunk start, with its first record out, before the lane before it gets there),
    // and an eighth when the call's lanes fill the chip (the warm-up is then extra work, not
    // idle time): RjCoefBuf.warm_shift.
    const uint32_t warm = (chunk && c > 0 && !empty)
                              ? min(b0, min(uint32_t(RJ_CHUNK_WARM_BYTES), (clen >> coefs.warm_shift) & ~15u))
                              : 0u;
    const uint32_t bs = b0 - warm;  // 16-B aligned: b0 and the warm-up both are
    const uint32_t lane_bytes = empty ? 0u : nbytes - bs;  // the lane may read on to the data's end
    const uint4 *src = reinterpret_cast<const uint4 *>(destuffed + im.destuff_off + sg.dst_off + bs);
    const uint32_t nchunks = (lane_bytes + 15) / 16;
    const HCol<DEC> ring{&s_ring[0][L]};

    if (mover) {  // the lean mover (k_huff)
      uint32_t cm = 0, na = 0;
      uint4 p0 = make_uint4(0, 0, 0, 0), p1 = p0, p2 = p0, p3 = p0;
      for (;;) {
        const uint32_t rd = lds_ld(&s_dec[L]);
        if (na > 0) {
          hl_put(ring, cm & (RJ_HL_CHUNKS - 1), p0);
          if (na > 1) hl_put(ring, (cm + 1) & (RJ_HL_CHUNKS - 1), p1);
          if (na > 2) hl_put(ring, (cm + 2) & (RJ_HL_CHUNKS - 1), p2);
          if (na > 3) hl_put(ring, (cm + 3) & (RJ_HL_CHUNKS - 1), p3);
          cm += na;
          lds_st(&s_mov[L], cm);
          na = 0;
        }
        const bool fin = rd == RJ_HL_FIN;
        const uint32_t live = fin ? RJ_HL_CHUNKS : cm - (rd >> 2);
        const uint32_t n = min(RJ_HL_CHUNKS - live, 4u);
        if (n > 0) {
          p0 = *gp(cm < nchunks ? src + cm : rj_hl_zero);
          if (n > 1) p1 = *gp(cm + 1 < nchunks ? src + cm + 1 : rj_hl_zero);
          if (n > 2) p2 = *gp(cm + 2 < nchunks ? src + cm + 2 : rj_hl_zero);
          if (n > 3) p3 = *gp(cm + 3 < nchunks ? src + cm + 3 : rj_hl_zero);
          na = n;
        }
        if (__builtin_amdgcn_ballot_w64(!fin) == 0) break;
        if (__builtin_amdgcn_ballot_w64(n > 0) == 0) __builtin_amdgcn_s_sleep(4);
      }
      continue;
    }

    // ---- decoder ----
    const uint32_t nblk = im.nblk_mcu;
    uint32_t pat = 0, cpat = 0;  // per block b (2 bits each): DC / AC table; component
    for (uint32_t bb = 0; bb < nblk; bb++) {
      const uint32_t cc = im.blk_comp[bb] & 3;
      pat |= ((im.comp_td[cc] & 1u) | ((im.comp_ta[cc] & 1u) << 1)) << (2 * bb);
      cpat |= cc << (2 * bb);
    }
    const uint32_t nb2 = 2 * nblk;
    const uint32_t pat_ac = pat >> 1;  // bit 2b: block b's AC table
    const uint32_t nbits = lane_bytes * 8u;  // data bits from the lane's first bit
    const uint32_t nbits_skip = chunk ? 0xFFFFFFFFu : nbits;  // chunk lanes never zero-fill (DONE instead)
    const uint32_t blocks = sg.mcu_count * nblk;
    const uint64_t ent_abs = im.ent_off + sg.ent_off;
    const uint32_t rcap = chunk ? uint32_t(rj_chunk_cap(rj_chunk_len(sg.src_len, nch))) : 0u;
    const uint64_t ent_lane = chunk ? gp(coefs.seg_ent)[gseg] + uint64_t(rj_chunk_lane(nch, H, c, h)) * rcap : ent_abs;
    uint32_t *ent = coefs.ent + ent_lane;
    const RjTableSet *tset = tabsets + T;
    const HCol<DEC> stage{&s_stage[0][L]};
    const uint32_t stage_a = lds_addr(&s_stage[0][L]), ring_a = lds_addr(&s_ring[0][L]);
    const uint32_t lut_a = lds_addr(s_lut), lut_dc = lut_a + RJ_HL_DC0;
    // chunk-lane state (rj_entropy.hip decode_lane)
    const uint32_t start_bit = bs * 8u, own_bit = b0 * 8u, end_bit = b1 * 8u, nbits_abs = nbytes * 8u;
    const uint32_t clen_bits = clen * 8u, ov_bit = end_bit + rj_chunk_reach(clen) * 8u;
    const uint32_t cap = rcap, next_chunks = chunk ? nch - 1 - c : 0u;
    const bool spec = chunk && c > 0;
    RjRecord *const rec_mine = coefs.rec + uint64_t(g) * RJ_MAX_RECORDS;
    // the records of chunk t, hypothesis hh: lane l_first + rj_chunk_lane(nch, H, t, hh)
    const RjRecord *const rec_int = coefs.rec + uint64_t(l_first) * RJ_MAX_RECORDS;
    uint32_t rb = 0, nrec = 0, tgt = 0, status = 0, rb_over = 0xFFFFFFFFu, s_tgt = 0, s_rec = 0;
    uint32_t next_tgt_bit = end_bit;
    uint32_t rec_rb = 0;  // blocks before the next record may be taken (its first: at the chunk start)
    // per hypothesis of the chunk being sought: the record looked at next, and the one loaded
    // at the phase start (key {pos, phase | epoch}, tagged with its (chunk, record))
    uint32_t j[NH], cache_tj[NH];
    uint64_t cache[NH];
#pragma unroll
    for (int hh = 0; hh < NH; hh++) {
      j[hh] = 0;
      cache_tj[hh] = 0xFFFFFFFFu;
      cache[hh] = 0;
    }
    bool rp = false;
    uint32_t rp_pos = 0, rp_b = 0, rp_ne = 0, rp_rb = 0;
    int rp_p0 = 0, rp_p1 = 0, rp_p2 = 0;
    int pred0 = 0, pred1 = 0, pred2 = 0;
    bool linked = false;  // kHyp: this lane's sync was published (s_link)
    const uint32_t wg_base = lane0 + blockIdx.x * DEC;
    if (empty) {
      RjChunkRes o = {};
      o.status = RJ_CHUNK_DONE;
      o.rb_over = 0xFFFFFFFFu;
      *gp(coefs.res + g) = o;
      hc_put_record<kScope>(rec_mine, 0xFFFFFFFFu, 0u, epoch, 0u, 0u, 0, 0, 0);
      lds_st(&s_dec[L], RJ_HL_FIN);
      continue;
    }
    if (spec && warm == 0) {  // no warm-up: the chunk's first bit is a block start by assumption (block h)
      hc_put_record<kScope>(rec_mine, start_bit, h, epoch, 0u, 0u, 0, 0, 0);
      nrec = 1;
      rec_rb = RJ_RECORD_EVERY;
    }
#define RJ_HC_WAIT_RING(upto)                                                                     \
  {                                                                                               \
    uint32_t cmv = lds_ld(&s_mov[L]);                                                             \
    while (__builtin_amdgcn_ballot_w64(4u * cmv < (upto)) != 0) {                                 \
      __builtin_amdgcn_s_sleep(2);                                                                \
      cmv = lds_ld(&s_mov[L]);                                                                    \
    }                                                                                             \
    avail = 4u * cmv;                                                                             \
    asm volatile("" ::: "memory");                                                                \
  }
    uint32_t avail = 0;
    RJ_HC_WAIT_RING(uint32_t(PHASE) + 2u);
#ifdef RJ_HL_STAMPS
    const uint64_t hc_t_loop = __builtin_amdgcn_s_memtime();
    hc_setup += hc_t_loop - hc_t_entry;
#endif
    uint32_t q = 0;
    uint32_t wa = 0, wb = ring[0], wc = ring[1];
    uint32_t rr = 1;
    uint32_t ne = 0, fl = 0;
    bool skip = !chunk && (sg.flags & RJ_SEG_MISSING) != 0;
    uint32_t blocks_left = chunk ? 0x7FFFFFFFu : blocks;
    uint32_t b = 2u * h, k = 0;  // a speculative lane starts in its hypothesis' phase (block h of an MCU)
    uint32_t acb = ((pat >> b >> 1) & 1u) * uint32_t(RJ_HL_AC_BYTES) + lut_a;  // LDS byte address
    uint32_t tb = RJ_HL_DC0 + (((pat >> b) & 1u) << (RJ_HL_DC_BITS + 2));
    uint32_t tsh = 32 - RJ_HL_DC_BITS;
    uint32_t peek = __builtin_amdgcn_alignbit(wa, wb, q);
    uint32_t e = s_lut[(tb >> 2) + (peek >> tsh)];
    while (__builtin_amdgcn_ballot_w64(blocks_left > 0) != 0) {
      if (blocks_left == 0) continue;
#ifdef RJ_HL_STAMPS
      const uint64_t hp0 = __builtin_amdgcn_s_memtime();
#endif
      // ---- phase start: the captured record leaves; the record being sought is loaded ----
      if (rp) {
        hc_put_record<kScope>(rec_mine + nrec, rp_pos, rp_b, epoch, rp_ne, rp_rb, rp_p0, rp_p1, rp_p2);
        nrec++;
        rp = false;
      }
      const uint32_t pos0 = start_bit + (0u - q);
      // lanes inside their own chunk (and exact lanes away from their end) cannot stop this phase
      const bool safe = __builtin_amdgcn_ballot_w64(
                            chunk ? pos0 + PHASE * 31u >= end_bit
                                  : !(blocks_left >= PHASE && !skip && (0u - q) + PHASE * 31u < nbits)) != 0;
      uint64_t rec_ld[NH];
      uint32_t rec_ld_tj[NH];
#pragma unroll
      for (int hh = 0; hh < NH; hh++) {
        rec_ld[hh] = 0;
        rec_ld_tj[hh] = 0xFFFFFFFFu;
      }
      const bool seek = chunk && pos0 + PHASE * 31u >= end_bit;
      if (__builtin_amdgcn_ballot_w64(seek) != 0) {
        const uint32_t t = tgt ? tgt : 1u;
#pragma unroll
        for (int hh = 0; hh < NH; hh++) {
          if (uint32_t(hh) < H) {
            const bool have = seek && t <= next_chunks && j[hh] < RJ_MAX_RECORDS;
            const RjRecord *r = have ? rec_int + uint64_t(rj_chunk_lane(nch, H, c + t, uint32_t(hh))) * RJ_MAX_RECORDS + j[hh]
                                     : rec_mine;
            rec_ld[hh] = __hip_atomic_load(reinterpret_cast<const uint64_t *>(r), __ATOMIC_RELAXED, kScope);
            rec_ld_tj[hh] = have ? (t << 16 | j[hh]) : 0xFFFFFFFFu;
          }
        }
      }
#ifdef RJ_HL_STAMPS
      const uint64_t hs0 = __builtin_amdgcn_s_memtime();
      hc_end[3] += hs0 - hp0;
#endif
      if (!safe) {
#pragma unroll
        for (uint32_t s_ = 0; s_ < PHASE; s_++) RJ_HC_STEP(false);
      } else {
#pragma unroll
        for (uint32_t s_ = 0; s_ < PHASE; s_++) RJ_HC_STEP(true);
      }
#ifdef RJ_HL_STAMPS
      const uint64_t hs1 = __builtin_amdgcn_s_memtime();
      if (safe) hc_safe_cyc += hs1 - hs0;
      else hc_uns_cyc += hs1 - hs0;
      hc_ph++;
      hc_safe += safe ? 1u : 0u;
#endif
      lds_st(&s_dec[L], max(rr, 2u) - 2u);
      if constexpr (kHyp && kScope == __HIP_MEMORY_SCOPE_WORKGROUP) {
        if (chunk && status == RJ_CHUNK_SYNC && !linked) {  // synced this phase: link, and pass the chain on
          linked = true;
          const uint32_t tl = l_first + rj_chunk_lane(nch, H, c + (s_tgt & 0xFFFFu), s_tgt >> 16) - wg_base;
          __hip_atomic_store(&s_link[L], tl, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (__hip_atomic_load(&s_onc[L], __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_WORKGROUP) != 0)
            hc_chain_walk(L, l_first - wg_base, nch, H, s_link, s_onc, s_conf);
        }
        if (chunk && c > 0 && status == 0 && start_bit + (0u - q) >= end_bit) {
          const uint32_t cf = __hip_atomic_load(&s_conf[L - h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (cf != 0u && cf != h + 1u) {  // another hypothesis of this chunk is on the chain
            status = RJ_CHUNK_FAIL;
            blocks_left = 0;
          }
        }
      }
#ifdef RJ_HL_STAMPS
      const uint64_t he1 = __builtin_amdgcn_s_memtime();
      hc_end[0] += he1 - hs1;
#endif
      // the records loaded at the phase start land here, before this phase's entry flush: a wait
      // for them placed after the flush would also wait for its stores (vmcnt counts loads and
      // stores in issue order)
#pragma unroll
      for (int hh = 0; hh < NH; hh++) {
        uint32_t lo = uint32_t(rec_ld[hh]), hi = uint32_t(rec_ld[hh] >> 32);
        asm volatile("" : "+v"(lo), "+v"(hi));
        cache[hh] = uint64_t(hi) << 32 | lo;
        cache_tj[hh] = rec_ld_tj[hh];
      }
#ifdef RJ_HL_STAMPS
      const uint64_t he2 = __builtin_amdgcn_s_memtime();
      hc_end[1] += he2 - he1;
#endif
      if (ne - fl >= GROUP) {
        hl_flush<DEC, GROUP>(stage, fl, ent + fl);
        fl += GROUP;
      }
#ifdef RJ_HL_STAMPS
      hc_end[2] += __builtin_amdgcn_s_memtime() - he2;
#endif
      if (__builtin_amdgcn_ballot_w64(avail < rr + PHASE + 1u) != 0) {
#ifdef RJ_HL_STAMPS
        const uint64_t hw0 = __builtin_amdgcn_s_memtime();
#endif
        RJ_HC_WAIT_RING(rr + PHASE + 1u);
        wc = ring[rr & (RJ_HL_WORDS - 1)];
#ifdef RJ_HL_STAMPS
        hc_wait += __builtin_amdgcn_s_memtime() - hw0;
#endif
      }
    }
#ifdef RJ_HL_STAMPS
    hc_loop += __builtin_amdgcn_s_memtime() - hc_t_loop;
#endif
#undef RJ_HC_WAIT_RING
    lds_st(&s_dec[L], RJ_HL_FIN);
    if (rp) hc_put_record<kScope>(rec_mine + nrec, rp_pos, rp_b, epoch, rp_ne, rp_rb, rp_p0, rp_p1, rp_p2);
    stage[ne & (kStage - 1)] = RJ_ENT_TERM;
    while (fl < ne + 1) {
      hl_flush<DEC, GROUP>(stage, fl, ent + fl);
      fl += GROUP;
    }
    if (chunk) {
      RjChunkRes o;
      o.status = status;
      o.tgt = s_tgt;  // chunks ahead | hypothesis << 16
      o.rec = s_rec;
      o.rb = rb;
      o.ne = ne;
      o.pred[0] = pred0;
      o.pred[1] = pred1;
      o.pred[2] = pred2;
      o.rb_over = rb_over;
      o.pad[0] = start_bit + (0u - q);
      o.pad[1] = end_bit;
      o.pad[2] = 0;
      *gp(coefs.res + g) = o;
    } else {
      *gp(coefs.piece + rj_seg_lane0(coefs, gseg)) = RjPiece{ent_abs, 0u, blocks, 1u, {0, 0, 0}};
    }
    if (coefs.count) atomicAdd(&s_ne, ne + 1);
  }
  if (tid == 0 && coefs.count != nullptr && s_ne != 0) atomicAdd(coefs.count, (unsigned long long)s_ne);
#ifdef RJ_HL_STAMPS
  if (!mover && (tid & 63) == 0 && hc_ph) {
    atomicAdd(&rj_hc_stamp[0], (unsigned long long)hc_setup);
    atomicAdd(&rj_hc_stamp[1], (unsigned long long)hc_loop);
    atomicAdd(&rj_hc_stamp[2], (unsigned long long)hc_ph);
    atomicAdd(&rj_hc_stamp[3], (unsigned long long)hc_safe);
    atomicAdd(&rj_hc_stamp[4], 1ull);
    atomicMax(&rj_hc_stamp[5], (unsigned long long)hc_loop);
    atomicAdd(&rj_hc_stamp[6], (unsigned long long)hc_wait);
    atomicMax(&rj_hc_stamp[7], (unsigned long long)(__builtin_amdgcn_s_memtime() - hc_t_entry));
    atomicAdd(&rj_hc_stamp[8], (unsigned long long)hc_safe_cyc);
    atomicAdd(&rj_hc_stamp[9], (unsigned long long)hc_uns_cyc);
    for (int q = 0; q < 4; q++) atomicAdd(&rj_hc_stamp[10 + q], (unsigned long long)hc_end[q]);
  }
#endif
}

hipError_t LaunchHuffChunks(hipStream_t st, const RjImageDev *imgs, int nimg, uint32_t lane0, uint32_t lanes_wg,
                            uint32_t lanes_dev, const uint8_t *destuffed, const RjTableSet *tabsets,
                            const RjLeanTables *lean, RjCoefBuf coefs, uint32_t epoch) {
  const bool hyp = coefs.hyp > 1;
  if (lanes_wg) {
    const dim3 grid((lanes_wg + RJ_K1_WG - 1) / RJ_K1_WG), block(2 * RJ_K1_WG);
    if (hyp)
      hipLaunchKernelGGL((k_huff_chunk<__HIP_MEMORY_SCOPE_WORKGROUP, true>), grid, block, 0, st, imgs, nimg, lane0,
                         lanes_wg, destuffed, tabsets, lean, coefs, epoch);
    else
      hipLaunchKernelGGL((k_huff_chunk<__HIP_MEMORY_SCOPE_WORKGROUP, false>), grid, block, 0, st, imgs, nimg, lane0,
                         lanes_wg, destuffed, tabsets, lean, coefs, epoch);
  }
  if (lanes_dev) {
    const dim3 grid((lanes_dev + RJ_K1_WG - 1) / RJ_K1_WG), block(2 * RJ_K1_WG);
    if (hyp)
      hipLaunchKernelGGL((k_huff_chunk<__HIP_MEMORY_SCOPE_AGENT, true>), grid, block, 0, st, imgs, nimg,
                         lane0 + lanes_wg, lanes_dev, destuffed, tabsets, lean, coefs, epoch);
    else
      hipLaunchKernelGGL((k_huff_chunk<__HIP_MEMORY_SCOPE_AGENT, false>), grid, block, 0, st, imgs, nimg,
                         lane0 + lanes_wg, lanes_dev, destuffed, tabsets, lean, coefs, epoch);
  }
  return hipGetLastError();
}

#ifdef RJ_HL_STAMPS
void DumpHuffStamps() {
  unsigned long long h[11];
  (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(rj_hl_stamp), sizeof(h));
  const double w = h[4] ? double(h[4]) : 1.0;
  const double ph = double(h[2] + h[3]) ? double(h[2] + h[3]) : 1.0;
  fprintf(stderr, "[rj k_huff] waves %llu: per wave %.0f phases (%.0f safe), %.0f escape steps; cycles per phase: steps %.0f, end %.0f; "
          "decode cycles per wave %.0f (max %llu); clock %.0f MHz; of the end: to the flush's end %.0f, ring checks per phase %.3f\n",
          h[4], ph / w, h[3] / w, h[5] / w, h[0] / ph, h[1] / ph, h[6] / w, h[7], h[8] ? 100.0 * double(h[6]) / double(h[8]) : 0.0,
          h[9] / ph, h[10] / ph);
  // (a stamp waits for the wave's outstanding LDS operations: "end" includes the drain of the
  // last steps' lookups, not only the phase-end work)
  unsigned long long z[11] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(rj_hl_stamp), z, sizeof(z));
  unsigned long long c[14];
  (void)hipMemcpyFromSymbol(c, HIP_SYMBOL(rj_hc_stamp), sizeof(c));
  if (c[4]) {
    const double wv = double(c[4]), pp = c[2] ? double(c[2]) : 1.0;
    fprintf(stderr, "[rj k_huff_chunk] decoder waves %llu: per wave setup %.0f cycles, loop %.0f (max %llu, wave max %llu from entry), "
            "%.0f phases (%.0f safe), %.0f cycles per phase, ring waits %.0f per wave; step cycles per safe phase %.0f, "
            "per other phase %.0f\n",
            c[4], c[0] / wv, c[1] / wv, c[5], c[7], c[2] / wv, c[3] / wv, c[1] / pp, c[6] / wv,
            c[3] ? double(c[8]) / double(c[3]) : 0.0, c[2] > c[3] ? double(c[9]) / double(c[2] - c[3]) : 0.0);
    fprintf(stderr, "[rj k_huff_chunk] per phase: s_dec + chain %.0f, record settle %.0f, flush %.0f, phase start %.0f cycles\n",
            c[10] / pp, c[11] / pp, c[12] / pp, c[13] / pp);
    unsigned long long z2[14] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(rj_hc_stamp), z2, sizeof(z2));
  }
}
#endif

hipError_t LaunchHuffLanes(hipStream_t st, const RjImageDev *imgs, int nimg, uint32_t lane0, uint32_t nlanes,
                           const uint8_t *destuffed, const RjTableSet *tabsets, const RjLeanTables *lean,
                           RjCoefBuf coefs, uint32_t extra_lds, const RjHuffSplit *split, bool five_waves,
                           const RjLive *live) {
  if (nlanes == 0) return hipSuccess;
  const RjLive lv = live != nullptr ? *live : RjLive{};
  if (split != nullptr && five_waves) {  // five-wave layout with split pairs first
    hipLaunchKernelGGL((k_huff<RJ_HL_DEC5, RJ_HL_GROUP, true, RJ_HL_PHASE>), dim3((nlanes + RJ_HL_DEC5 - 1) / RJ_HL_DEC5),
                       dim3(2 * RJ_HL_DEC5), 0, st, imgs, nimg, lane0, nlanes, destuffed, tabsets, lean, coefs, *split, lv);
  } else if (split != nullptr) {  // outliers split: one decoder wave per SIMD, two workgroups per CU
    hipLaunchKernelGGL((k_huff<RJ_HL_SPLIT_DEC, 8, true, 4>), dim3((nlanes + RJ_HL_SPLIT_DEC - 1) / RJ_HL_SPLIT_DEC),
                       dim3(2 * RJ_HL_SPLIT_DEC), 0, st, imgs, nimg, lane0, nlanes, destuffed, tabsets, lean, coefs,
                       *split, lv);
  } else {
    if (five_waves)  // one workgroup per CU by its LDS (~105 KB)
      hipLaunchKernelGGL((k_huff<RJ_HL_DEC5, RJ_HL_GROUP, false, RJ_HL_PHASE>),
                         dim3((nlanes + RJ_HL_DEC5 - 1) / RJ_HL_DEC5), dim3(2 * RJ_HL_DEC5), 0, st, imgs, nimg, lane0,
                         nlanes, destuffed, tabsets, lean, coefs, RjHuffSplit{0, 0}, lv);
    else
      hipLaunchKernelGGL((k_huff<256, RJ_HL_GROUP, false, RJ_HL_PHASE>), dim3((nlanes + 255) / 256), dim3(512),
                         extra_lds, st, imgs, nimg, lane0, nlanes, destuffed, tabsets, lean, coefs, RjHuffSplit{0, 0}, lv);
  }
  return hipGetLastError();
}

}  // namespace rj
