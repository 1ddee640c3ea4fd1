// rj_entropy.hip -- K1: baseline Huffman entropy decode (T.81 F.2.2, libjpeg jdhuff.c semantics).
//
// The reference hands this step to VCN (src/rocjpeg_vaapi_decoder.cpp:677-689).  Here every
// restart interval is decoded by one or more lanes:
//
//   * short intervals (< RJ_SPLIT_BYTES): one lane, exact serial semantics --
//     libjpeg's "insufficient data" rule (the MCU that runs past the data is decoded with zero
//     bits, the rest of the interval is zero) and missing-RST intervals;
//   * long intervals (long DRI, or no DRI at all -- every reference fixture): one lane per
//     chunk.  Chunk 0 starts in the true state; chunk c > 0 starts speculatively at its first
//     bit, as if a Y block began there, and records its state at every 4th block start of its
//     head.  Huffman codes self-synchronise: a lane that runs past its own end compares its
//     (true) state at each block start with the records of the chunk it has entered and stops
//     at the first equal state -- from there on both decodes are identical.  k_resolve chains
//     the sync points into pieces (which part of which chunk stream holds which blocks, and
//     the DC-predictor correction of each piece); an interval whose chunks did not sync within
//     rj_chunk_reach, or whose data ends before its blocks (truncated stream), is decoded
//     again serially by k_entropy<true>.  Chunks are laid out in reverse order over the lanes,
//     so the chunk a lane has to read records from was dispatched no later than itself.
//
// Per lane everything on the per-symbol dependency chain stays on-chip:
//   * bits: 64-bit MSB-first buffer refilled 32 bits at a time from a per-lane LDS ring of the
//     destuffed bytes (read one symbol ahead); the ring is topped up from HBM at wave-uniform
//     phase boundaries with loads issued one phase before they are committed -- the symbol
//     loop itself never reads HBM (a conditional global load there costs a vmcnt(0) round trip);
//   * lookup: two-level LUT in LDS (9-bit first level + 7-bit second level, rj_device.h), one
//     copy per workgroup of 4 waves; the extra bits come from the same 32-bit peek;
//   * output: per-lane LDS stage, 64-B groups written at phase boundaries.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "rj_device.h"
#include "rj_kernels.h"
#include "rj_math.h"

namespace rj {

#define RJ_RING_CHUNKS 6   // 16-B chunks per lane in the bit ring (96 B)
#define RJ_RING_WORDS (RJ_RING_CHUNKS * 4)
#define RJ_PHASE 8         // symbols per phase: <= 8 ring words consumed (<= 31 bits/symbol)
#define RJ_PREFETCH 2      // chunks fetched per phase at most
#define RJ_STAGE 32        // staged entries per lane (two 64-B groups)
#define RJ_WG 256          // 4 waves share one LDS copy of the tables
// Ring invariant: after every phase commit the ring holds >= 8 unread words (or all that is
// left).  With U unread words a phase prefetches n = min(2, 6 - used) chunks and consumes at
// most 8 words: U >= 16 keeps U' >= 8; 8 <= U < 16 means used <= 4, so n = 2 and U' = U.

// One lane's column of a lane-interleaved LDS array: word w of lane l at [w][l], so that the
// lanes' private rings and stages sit in distinct banks whatever word each lane touches.
struct LRow {
  uint32_t *base;  // &array[0][lane]
  __device__ __forceinline__ uint32_t &operator[](uint32_t w) const { return base[w * RJ_WG]; }
};

// one 64-B group of staged entries (16 words from slot `from`, a multiple of 16) to HBM
__device__ __forceinline__ void flush_group(const LRow &stage, uint32_t from, uint32_t *dst) {
  uint32_t w[RJ_ENT_GROUP];
#pragma unroll
  for (int q = 0; q < RJ_ENT_GROUP; q++) w[q] = stage[(from & (RJ_STAGE - 1)) + q];
  uint4 *d4 = reinterpret_cast<uint4 *>(dst);
#pragma unroll
  for (int q = 0; q < RJ_ENT_GROUP / 4; q++) gp(d4)[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

struct BitReader {
  const uint4 *src;   // 16-B aligned destuffed bytes (from the lane's start), zero-padded
  LRow ring;          // this lane's LDS ring (RJ_RING_WORDS words)
  uint32_t nchunks;   // 16-B chunks holding data
  uint32_t rd;        // words moved into the bit buffer (monotonic)
  uint32_t rdw;       // rd mod RJ_RING_WORDS
  uint32_t cm;        // chunks committed to the ring (monotonic)
  uint32_t cms;       // cm mod RJ_RING_CHUNKS
  uint32_t nw;        // ring word rd, read ahead
  int nb;             // valid bits in acc (left-justified)
  uint64_t acc;

  __device__ __forceinline__ void init(const uint4 *s, LRow r, uint32_t nbytes) {
    src = s;
    ring = r;
    nchunks = (nbytes + 15) / 16;
    const uint32_t first = nchunks < RJ_RING_CHUNKS ? nchunks : RJ_RING_CHUNKS;
    for (uint32_t q = 0; q < first; q++) put4(q, gp(src)[q]);
    cm = first;
    cms = first == RJ_RING_CHUNKS ? 0 : first;
    rd = 0;
    rdw = 0;
    nw = ring[0];
    nb = 0;
    acc = 0;
  }
  // Phase start: issue the loads of up to RJ_PREFETCH chunks (unconditional, clamped: a
  // conditional load would force an immediate wait).  Phase end: commit them to the ring.
  // The loaded registers live only inside one phase (no loop-carried copy of an in-flight
  // load, which would make the compiler wait for it at once).
  __device__ __forceinline__ uint32_t issue(uint4 &pf0, uint4 &pf1) const {
    static_assert(RJ_PREFETCH == 2, "two prefetch registers");
    const uint32_t used = cm - (rd >> 2);  // live chunks, incl. the one being read
    const uint32_t room = RJ_RING_CHUNKS - used;
    uint32_t want = nchunks > cm ? nchunks - cm : 0u;
    want = want < room ? want : room;
    const uint32_t n = want < RJ_PREFETCH ? want : RJ_PREFETCH;
    const uint32_t last = nchunks ? nchunks - 1 : 0;
    pf0 = gp(src)[cm < last ? cm : last];
    pf1 = gp(src)[cm + 1 < last ? cm + 1 : last];
    return n;
  }
  __device__ __forceinline__ void put4(uint32_t slot, const uint4 &v) {
    ring[4 * slot] = v.x;
    ring[4 * slot + 1] = v.y;
    ring[4 * slot + 2] = v.z;
    ring[4 * slot + 3] = v.w;
  }
  __device__ __forceinline__ void commit(const uint4 &pf0, const uint4 &pf1, uint32_t n) {
    if (n > 0) {
      put4(cms, pf0);
      cms = cms == RJ_RING_CHUNKS - 1 ? 0 : cms + 1;
    }
    if (n > 1) {
      put4(cms, pf1);
      cms = cms == RJ_RING_CHUNKS - 1 ? 0 : cms + 1;
    }
    cm += n;
    nw = ring[rdw];  // the commit may have landed the read-ahead word
  }
  __device__ __forceinline__ void refill() {  // branch-free
    const bool need = nb <= 32;
    const uint32_t w = (need && rd < 4 * cm) ? nw : 0u;  // past the data: zero bits, as libjpeg inserts
    acc |= uint64_t(__builtin_bswap32(w)) << ((32 - nb) & 63);
    nb += need ? 32 : 0;
    rd += need ? 1u : 0u;
    rdw = need ? (rdw == RJ_RING_WORDS - 1 ? 0 : rdw + 1) : rdw;
    nw = ring[rdw];
  }
  __device__ __forceinline__ uint32_t consumed() const { return rd * 32u - uint32_t(nb); }  // bits
};

// canonical search for codes the LDS tables do not resolve (second-level pool exhausted, or a
// DC code longer than 9 bits): libjpeg jpeg_huff_decode on the table in HBM
__device__ __forceinline__ uint32_t huff_slow(const RjHuffDev *t, uint32_t peek16) {
  uint32_t e = RJ_LUT_BAD;
#pragma unroll 1
  for (int l = 1; l <= 16; l++)  // a loop: rare path, kept small in the unrolled symbol loop
    if (peek16 < t->maxcode16[l]) {
      e = uint32_t(l << 8) | t->vals[((peek16 >> (16 - l)) + t->valoff[l]) & 255];
      break;
    }
  return e;
}

// LDS table image: DC tables first level only (512 entries each), AC tables both levels
#define RJ_SLUT_AC0 (2 * RJ_LUT_L1)
#define RJ_SLUT_ENTRIES (2 * RJ_LUT_L1 + 2 * RJ_LUT_ENTRIES)

__device__ __forceinline__ uint64_t rec_key(uint32_t pos, uint32_t b, uint32_t epoch) {
  return uint64_t(pos) | (uint64_t((b & 15u) | (epoch << 4)) << 32);
}
// Publish a chunk-start record.  The reader only looks at the 8-B key {pos, tag}; k_resolve
// reads the rest after the kernel.  Workgroup scope: one 16-B store into the CU's coherent
// cache level; agent scope: the key as a device-coherent atomic.
template <int kScope>
__device__ __forceinline__ void put_record(RjRecord *r, uint32_t pos, uint32_t b, uint32_t epoch, uint32_t ne,
                                           uint32_t rb, int p0, int p1, int p2) {
  *gp(reinterpret_cast<int4 *>(&r->pred[0])) = make_int4(p0, p1, p2, 0);
  if (kScope == __HIP_MEMORY_SCOPE_WORKGROUP) {
    *gp(reinterpret_cast<uint4 *>(r)) = make_uint4(pos, (b & 15u) | (epoch << 4), ne, rb);
  } else {
    *gp(reinterpret_cast<uint2 *>(&r->ne)) = make_uint2(ne, rb);
    __hip_atomic_store(reinterpret_cast<uint64_t *>(r), rec_key(pos, b, epoch), __ATOMIC_RELAXED, kScope);
  }
}

// The decode of one lane.  kSplit: speculative/seek chunk of a long interval (stops at a sync
// point or the end of the data); else exact serial decode of a whole interval.
struct LaneJob {
  const uint4 *src;    // destuffed bytes from the lane's first byte
  uint32_t bytes;      // bytes available from there to the end of the interval's data
  uint32_t start_bit;  // interval bit position of the lane's first bit
  uint32_t end_bit;    // interval bit position where the lane's own chunk ends (split)
  uint32_t ov_bit;     // give-up point (split)
  uint32_t nbits;      // interval data bits
  uint32_t blocks;     // exact: blocks of the interval
  uint32_t *ent;       // the lane's entry region
  uint32_t cap;        // its capacity (split)
  bool missing;        // exact: RST marker missing -> all blocks zero
  bool spec;           // split, c > 0: write chunk-start records
  RjRecord *rec;       // this chunk's records
  const RjRecord *rec_next;  // records of chunk c+1 (chunk c+t at rec_next - (t-1) lanes: reverse order)
  uint32_t next_chunks;      // chunks after this one
  uint32_t clen_bits;
  // exact lanes: pieces at MCU-row checkpoints, so that K2 finds any row without a long skip
  RjPiece *pieces;     // the interval's piece slots
  uint32_t slots;      // how many
  uint64_t ent_abs;    // absolute entry index of J.ent
  uint32_t mcux, mcu_first, mcu_count;
};

// empty asm with a read-write VGPR operand: the value is computed unconditionally before it,
// which keeps selects on it as v_cndmask (otherwise the structurizer may sink each operand's
// computation into its own branch, with the exec-mask SALU that brings)
__device__ __forceinline__ void opaque(uint32_t &v) { asm volatile("" : "+v"(v)); }

// 32 zero bytes: what the exact decoder reads past the end of an interval's data
__device__ const uint4 rj_zero_chunks[RJ_PREFETCH] = {};

// Exact serial decode of one whole interval (one lane).  Every lane of the wave runs the same
// number of symbol steps per phase (no per-lane loop exit: a lane that has finished its blocks
// keeps stepping with its effects masked), and the per-symbol bookkeeping is select-only, so
// the loop carries no exec-mask juggling.
// Bits: a 32-word LDS ring (+ a mirror of word 0 at index 32) of big-endian stream words.  The
// words i = pos >> 5 and i + 1 sit in registers and a 64-bit shift by pos & 31 gives the
// 32-bit peek; word i + 2 is read one step ahead, so a step that crosses a word boundary
// shifts registers instead of waiting on the ring (off the symbol dependency chain).  Chunks are byte-swapped
// once, when they land in the ring; past the data the ring receives zero chunks (the zero
// bits libjpeg inserts).  Ring invariant: >= 8 unread words at every phase start (a phase
// reads <= 8: 8 symbols of <= 27 bits plus the next word); with U unread words a phase
// commits n = min(2, 8 - live chunks) chunks and reads <= 7: U >= 16 keeps U' >= 9, and
// 8 <= U < 16 means <= 4 live chunks, so n = 2 and U' >= U + 1.
// kCkpt: MCU-row checkpoint pieces (the serial fallback of long intervals); the main pass's
// exact lanes have one piece slot and skip that bookkeeping.
#define RJ_XRING_CHUNKS 8
#define RJ_XRING_WORDS (RJ_XRING_CHUNKS * 4)

__device__ __forceinline__ void xring_put(const LRow &ring, uint32_t slot, const uint4 &v) {
  const uint32_t w0 = __builtin_bswap32(v.x), w1 = __builtin_bswap32(v.y);
  const uint32_t w2 = __builtin_bswap32(v.z), w3 = __builtin_bswap32(v.w);
  ring[4 * slot] = w0;
  ring[4 * slot + 1] = w1;
  ring[4 * slot + 2] = w2;
  ring[4 * slot + 3] = w3;
  if (slot == 0) ring[RJ_XRING_WORDS] = w0;  // mirror: word 31's successor
}

// One symbol step of decode_exact (SAFE: per-lane activity mask and insufficient-data handling).
#define RJ_EXACT_STEP(SAFE) \
  do { \
      const bool act = !(SAFE) || blocks_left > 0; \
      const uint32_t peek32 = uint32_t((((uint64_t(w0) << 32) | w1) << (pos & 31)) >> 32); \
      const bool isdc = k == 0; \
      uint32_t e = s_lut[tbase + (peek32 >> 23)]; \
      if (e & 0x8000u) { \
        if (e != 0xFFFFu && !isdc) { \
          e = s_lut[tbase + RJ_LUT_L1 + (e & 0x7Fu) * 128u + ((peek32 >> 16) & 127u)]; \
        } else { \
          const RjHuffDev *t = isdc ? &ts->dc[(info >> 2) & 1u] : &ts->ac[(info >> 3) & 1u]; \
          e = huff_slow(t, peek32 >> 16); \
        } \
      } \
      const uint32_t len = e >> 8, sym = e & 255u; \
      const uint32_t sz = sym & 15u, r = sym >> 4; \
      const uint32_t raw = __builtin_amdgcn_ubfe(peek32, 32u - len - sz, sz); \
      const int val = int(raw) + (int32_t(raw - (1u << ((sz - 1) & 31))) >> 31 & int32_t(1u - (1u << sz))); \
      { /* words i, i+1 in w0, w1; word i+2 (read one step ahead) in w2 */ \
        const uint32_t npos = pos + len + sz; \
        const bool adv = (npos >> 5) != (pos >> 5); \
        w0 = adv ? w1 : w0; \
        w1 = adv ? w2 : w1; \
        w2 = ring[((npos >> 5) + 2) & (RJ_XRING_WORDS - 1)]; \
        pos = npos; \
      } \
      const uint32_t c = info & 3u; \
      const int p = (c == 0 ? pred0 : (c == 1 ? pred1 : pred2)) + val; \
      pred0 = (isdc && c == 0) ? p : pred0; \
      pred1 = (isdc && c == 1) ? p : pred1; \
      pred2 = (isdc && c == 2) ? p : pred2; \
      const uint32_t kk = isdc ? 0u : k + r;  /* zigzag position of this coefficient */ \
      /* AC: EOB (size 0, run != 15) ends the block; ZRL and coefficients advance k to kk + 1 */ \
      const bool eob = !isdc && sz == 0 && r != 15; \
      uint32_t entry = (uint32_t(isdc ? p : val) & 0xFFFFu) | (min(kk, 63u) << 16); \
      bool emit = isdc || sz != 0; \
      uint32_t knew = kk + 1u; \
      opaque(knew); \
      knew = eob ? 64u : knew; \
      if (SAFE) { \
        entry = skip ? 0u : entry;  /* libjpeg: the rest of the interval decodes to zero blocks */ \
        emit = skip || emit; \
        knew = skip ? 64u : knew; \
      } \
      stage[ne & (RJ_STAGE - 1)] = entry;  /* a non-emitted write lands in the next free slot */ \
      ne += (emit && act) ? 1u : 0u; \
      const bool bend = knew >= 64u; \
      const uint32_t bn = b + 1 == nblk ? 0u : b + 1; \
      const bool mcuend = bend && bn == 0; \
      k = bend ? 0u : knew; \
      b = bend ? bn : b; \
      info = uint32_t(binfo >> (4 * b)) & 15u; \
      acbase = RJ_SLUT_AC0 + ((info >> 3) & 1u) * RJ_LUT_ENTRIES; \
      uint32_t dcb = ((info >> 2) & 1u) * RJ_LUT_L1; \
      opaque(dcb);  /* both operands materialised: the select stays a v_cndmask, not a branch */ \
      opaque(acbase); \
      tbase = bend ? dcb : acbase; \
      blocks_left -= (bend && act) ? 1u : 0u; \
      if (SAFE) skip = skip || (mcuend && pos > J.nbits); \
      if (kCkpt) { \
        to_row -= (mcuend && act) ? 1u : 0u; \
        if (to_row == 0) {  /* the next MCU starts a row (rare) */ \
          to_row = J.mcux; \
          if (--rows_left == 0) { \
            rows_left = every; \
            if (blocks_left && np < J.slots) {  /* checkpoint: a new piece starts here */ \
              const uint32_t bdone = J.blocks - blocks_left; \
              gp(J.pieces + np - 1)->nblk = bdone - pfirst; \
              *gp(J.pieces + np) = RjPiece{J.ent_abs + ne, bdone, 0u, 0u, {0, 0, 0}}; \
              pfirst = bdone; \
              np++; \
            } \
          } \
        } \
      } \
     \
  } while (0)

template <bool kCkpt>
__device__ __forceinline__ uint32_t decode_exact(const LaneJob &J, uint64_t binfo, uint32_t nblk, const uint16_t *s_lut,
                                             const RjTableSet *ts, LRow ring, LRow stage) {
  const uint4 *src = J.src;
  const uint32_t nchunks = (J.bytes + 15) / 16;
  for (uint32_t q = 0; q < RJ_XRING_CHUNKS; q++)
    xring_put(ring, q, *gp(q < nchunks ? src + q : rj_zero_chunks));
  uint32_t cm = RJ_XRING_CHUNKS;  // chunks committed (past the data: zero chunks)
  uint32_t pos = 0;               // bits consumed
  uint32_t w0 = ring[0], w1 = ring[1], w2 = ring[2];
  uint32_t ne = 0, fl = 0;
  int pred0 = 0, pred1 = 0, pred2 = 0;
  bool skip = J.missing;
  uint32_t blocks_left = J.blocks;
  uint32_t b = 0;
  uint32_t info = uint32_t(binfo) & 15u;
  uint32_t acbase = RJ_SLUT_AC0 + ((info >> 3) & 1u) * RJ_LUT_ENTRIES;
  uint32_t tbase = ((info >> 2) & 1u) * RJ_LUT_L1;  // table of the next symbol (DC of block 0)
  uint32_t k = 0;
  // row checkpoints every `every` MCU rows of the interval (piece slots permitting)
  uint32_t np = 1, pfirst = 0, to_row = 0, rows_left = 0, every = 1;
  if (kCkpt) {
    const uint32_t r0 = J.mcu_first / J.mcux;
    const uint32_t rows = (J.mcu_first + J.mcu_count - 1) / J.mcux - r0 + 1;
    every = (rows + J.slots - 1) / J.slots;
    to_row = J.mcux - (J.mcu_first - r0 * J.mcux);  // MCUs until the next row starts
    rows_left = every;
  }
  // Prefetch issued at the end of a phase (after that phase's stage flush) lands in the ring at
  // the end of the next one: the wait for it then also covers the flush stores (vmcnt counts
  // stores too, in issue order), which have had a whole phase to complete.
  uint32_t n = 0;  // chunks in flight (issued at the end of the previous phase)
  uint4 pf0 = make_uint4(0, 0, 0, 0), pf1 = make_uint4(0, 0, 0, 0);
  while (__builtin_amdgcn_ballot_w64(blocks_left > 0) != 0) {
    // A phase in which no lane can finish its blocks or reach the end of its data (each step
    // ends at most one block and reads at most 31 bits) needs neither the per-lane activity
    // mask nor libjpeg's insufficient-data handling: that body is the common one.
    const bool fast = !kCkpt && __builtin_amdgcn_ballot_w64(!(blocks_left >= RJ_PHASE && !skip &&
                                                              pos + RJ_PHASE * 31u < J.nbits)) == 0;
    if (fast) {
#pragma unroll
      for (uint32_t q = 0; q < RJ_PHASE; q++) RJ_EXACT_STEP(false);
    } else {
#pragma unroll
      for (uint32_t q = 0; q < RJ_PHASE; q++) RJ_EXACT_STEP(true);
    }
    // ---- phase end (wave-uniform): the previous prefetch lands in the ring, a full stage
    // group leaves, the next prefetch is issued (zero chunks past the data) ----
    if (n > 0) xring_put(ring, cm & (RJ_XRING_CHUNKS - 1), pf0);
    if (n > 1) xring_put(ring, (cm + 1) & (RJ_XRING_CHUNKS - 1), pf1);
    cm += n;
    // the last step's read-ahead word may predate this commit (words i, i+1 never do: >= 9
    // unread words were committed at the phase start)
    w2 = ring[((pos >> 5) + 2) & (RJ_XRING_WORDS - 1)];
    if (ne - fl >= RJ_ENT_GROUP) {
      flush_group(stage, fl, J.ent + fl);
      fl += RJ_ENT_GROUP;
    }
    n = min(RJ_XRING_CHUNKS - (cm - (pos >> 7)), 2u);  // slots free now stay free until it lands
    pf0 = *gp(cm < nchunks ? src + cm : rj_zero_chunks);
    pf1 = *gp(cm + 1 < nchunks ? src + cm + 1 : rj_zero_chunks + 1);
  }
  stage[ne & (RJ_STAGE - 1)] = RJ_ENT_TERM;
  while (fl < ne + 1) {
    flush_group(stage, fl, J.ent + fl);
    fl += RJ_ENT_GROUP;
  }
  gp(J.pieces + np - 1)->nblk = J.blocks - pfirst;
  gp(J.pieces)->npieces = np;
  return ne + 1;  // entries incl. the terminator
}

template <bool kSplit, int kScope>
__device__ __forceinline__ uint32_t decode_lane(const LaneJob &J, uint64_t binfo, uint32_t nblk, uint32_t epoch,
                                            const uint16_t *s_lut, const RjTableSet *ts, LRow ring,
                                            LRow stage, RjChunkRes *res) {
  BitReader br;
  br.init(J.src, ring, J.bytes);
  uint32_t ne = 0, fl = 0;  // entries produced / flushed (fl multiple of RJ_ENT_GROUP)
  int pred0 = 0, pred1 = 0, pred2 = 0;
  bool skip = J.missing;
  uint32_t blocks_left = kSplit ? 0xFFFFFFFFu : J.blocks;
  uint32_t b = 0;
  uint32_t info = uint32_t(binfo) & 15u;
  uint32_t dcbase = ((info >> 2) & 1u) * RJ_LUT_L1, acbase = RJ_SLUT_AC0 + ((info >> 3) & 1u) * RJ_LUT_ENTRIES;
  int k = 0;
  // split-lane state
  uint32_t rb = 0;                 // blocks completed
  uint32_t nrec = 0;
  uint32_t tgt = 0, j = 0;         // chunk (relative to this one, 1-based) and record being sought
  uint64_t cache = 0;              // record key of (tgt, j), loaded during the previous phase
  uint32_t cache_tj = 0xFFFFFFFFu;
  uint32_t status = 0, rb_over = 0xFFFFFFFFu, s_tgt = 0, s_rec = 0;
  uint32_t next_tgt_bit = J.end_bit;  // where the next later chunk begins
  // exact lanes: row checkpoints every `every` MCU rows of the interval (piece slots permitting)
  uint32_t to_row = 0, rows_left = 0, every = 1, np = 1, pfirst = 0, bdone = 0;
  if (!kSplit) {
    const uint32_t r0 = J.mcu_first / J.mcux;
    const uint32_t rows = (J.mcu_first + J.mcu_count - 1) / J.mcux - r0 + 1;
    every = (rows + J.slots - 1) / J.slots;
    to_row = J.mcux - (J.mcu_first - r0 * J.mcux);  // MCUs until the next row starts
    rows_left = every;
  }
  if (kSplit && J.spec) {
    put_record<kScope>(J.rec, J.start_bit, 0u, epoch, 0u, 0u, 0, 0, 0);
    nrec = 1;
  }
  // a record taken mid-phase is stored at the next phase start: a store issued inside the
  // symbol loop would hold up the phase-end wait for the prefetch (vmcnt counts stores too).
  // Records are >= 8 blocks (>= 16 symbols, two phases) apart, so one register copy suffices.
  bool rp = false;
  uint32_t rp_pos = 0, rp_b = 0, rp_ne = 0, rp_rb = 0;
  int rp_p0 = 0, rp_p1 = 0, rp_p2 = 0;
  while (kSplit ? status == 0 : blocks_left > 0) {
    // ---- phase start (same count in every active lane): prefetch, record load, stage flush ----
    uint4 pf0, pf1;
    const uint32_t pn = br.issue(pf0, pf1);
    uint64_t rec_ld = 0;
    uint32_t rec_ld_tj = 0xFFFFFFFFu;
    if (kSplit) {  // record of the chunk being sought: compared from the next phase on
      const uint32_t t = tgt ? tgt : 1u;
      const bool have = t <= J.next_chunks && j < RJ_MAX_RECORDS;
      const RjRecord *r = have ? J.rec_next - int64_t(t - 1) * RJ_MAX_RECORDS + j : J.rec;
      rec_ld = __hip_atomic_load(reinterpret_cast<const uint64_t *>(r), __ATOMIC_RELAXED, kScope);
      rec_ld_tj = have ? (t << 16 | j) : 0xFFFFFFFFu;
    }
    if (kSplit && rp) {
      put_record<kScope>(J.rec + nrec, rp_pos, rp_b, epoch, rp_ne, rp_rb, rp_p0, rp_p1, rp_p2);
      nrec++;
      rp = false;
    }
    if (ne - fl >= RJ_ENT_GROUP) {  // one full 64-B group leaves the stage
      flush_group(stage, fl, J.ent + fl);
      fl += RJ_ENT_GROUP;
    }
    for (uint32_t step = 0; step < RJ_PHASE && (kSplit ? status == 0 : blocks_left > 0); step++) {
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
      const uint32_t tbase = k == 0 ? dcbase : acbase;
      uint32_t e = s_lut[tbase + (peek32 >> 23)];
      if (e & 0x8000u) {
        if (e != 0xFFFFu && k != 0) {
          e = s_lut[tbase + RJ_LUT_L1 + (e & 0x7Fu) * 128u + ((peek32 >> 16) & 127u)];
        } else {
          const RjHuffDev *t = k == 0 ? &ts->dc[(info >> 2) & 1u] : &ts->ac[(info >> 3) & 1u];
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
    // block / MCU bookkeeping as selects (lanes end blocks at different iterations)
    const bool bend = k >= 64;
    const uint32_t bn = b + 1 == nblk ? 0u : b + 1;
    const bool mcuend = bend && bn == 0;
    k = bend ? 0 : k;
    b = bend ? bn : b;
    info = uint32_t(binfo >> (4 * b)) & 15u;
    dcbase = ((info >> 2) & 1u) * RJ_LUT_L1;
    acbase = RJ_SLUT_AC0 + ((info >> 3) & 1u) * RJ_LUT_ENTRIES;
    if (!kSplit) {
      blocks_left -= bend ? 1u : 0u;
      bdone += bend ? 1u : 0u;
      // libjpeg: after an MCU that ran past the data the rest of the interval stays zero
      skip = skip || (mcuend && br.consumed() > J.nbits);
      to_row -= mcuend ? 1u : 0u;
      if (to_row == 0) {  // the next MCU starts a row (rare)
        to_row = J.mcux;
        if (--rows_left == 0) {
          rows_left = every;
          if (blocks_left && np < J.slots) {  // checkpoint: a new piece starts here
            gp(J.pieces + np - 1)->nblk = bdone - pfirst;
            *gp(J.pieces + np) = RjPiece{J.ent_abs + ne, bdone, 0u, 0u, {0, 0, 0}};
            pfirst = bdone;
            np++;
          }
        }
      }
    } else if (bend) {  // block start: records, sync search, stop conditions
      rb++;
      const uint32_t pos = J.start_bit + br.consumed();
      if (J.spec && nrec < RJ_MAX_RECORDS && rb % RJ_RECORD_EVERY == 0 && pos < J.end_bit) {
        rp = true;
        rp_pos = pos;
        rp_b = b;
        rp_ne = ne;
        rp_rb = rb;
        rp_p0 = pred0;
        rp_p1 = pred1;
        rp_p2 = pred2;
      }
      if (pos >= next_tgt_bit && tgt < J.next_chunks) {  // entered the next later chunk
        tgt++;
        j = 0;
        next_tgt_bit += J.clen_bits;
      }
      if (tgt) {  // records exist for the head of chunk c+tgt only
        if (cache_tj == (tgt << 16 | j) && uint32_t(cache >> 36) == (epoch & 0x0FFFFFFFu)) {
          const uint32_t cpos = uint32_t(cache);
          if (cpos == pos && uint32_t(cache >> 32 & 15u) == b) {
            status = RJ_CHUNK_SYNC;  // identical state from here on: the later chunk owns the rest
            s_tgt = tgt;
            s_rec = j;
          } else if (cpos < pos) {
            j++;
          }
        }
      }
      if (status == 0 && pos >= J.nbits) {  // end of the data
        if (pos > J.nbits) rb_over = rb - 1;
        status = RJ_CHUNK_DONE;
      }
      if (status == 0 && (pos > J.ov_bit || ne + 2 * RJ_ENT_PER_BLOCK > J.cap)) status = RJ_CHUNK_FAIL;
    }
    }
    // ---- phase end: the prefetch (one phase old) lands in the ring ----
    br.commit(pf0, pf1, pn);
    if (kSplit) {
      cache = rec_ld;
      cache_tj = rec_ld_tj;
    }
  }
  if (kSplit && rp) put_record<kScope>(J.rec + nrec, rp_pos, rp_b, epoch, rp_ne, rp_rb, rp_p0, rp_p1, rp_p2);
  // terminator, then everything still staged (whole groups; the slack is reserved)
  stage[ne & (RJ_STAGE - 1)] = RJ_ENT_TERM;
  while (fl < ne + 1) {
    flush_group(stage, fl, J.ent + fl);
    fl += RJ_ENT_GROUP;
  }
  if (!kSplit) {
    gp(J.pieces + np - 1)->nblk = bdone - pfirst;
    gp(J.pieces)->npieces = np;
  }
  if (kSplit) {
    RjChunkRes o;
    o.status = status;
    o.tgt = s_tgt;
    o.rec = s_rec;
    o.rb = rb;
    o.ne = ne;
    o.pred[0] = pred0;
    o.pred[1] = pred1;
    o.pred[2] = pred2;
    o.rb_over = rb_over;
    o.pad[0] = J.start_bit + br.consumed();  // stop position (diagnostics)
    o.pad[1] = J.end_bit;
    o.pad[2] = 0;
    *gp(res) = o;
  }
  return ne + 1;
}

// kFallback = false: one lane per chunk (all intervals).  kFallback = true: one lane per
// interval, only those k_resolve flagged, exact serial decode over the interval's regions.
// kFallback = false: one lane per chunk, lanes [lane0, lane0 + nlanes) of the call's lane
// layout (kScope: how records travel -- workgroup for intervals inside one workgroup, agent for
// the rest).  kFallback = true: one lane per interval, only those k_resolve flagged, exact
// serial decode over the interval's regions.
template <bool kFallback, int kScope>
__global__ __launch_bounds__(RJ_WG, 2) void k_entropy(const RjImageDev *__restrict__ imgs, int nimg, uint32_t lane0,
                                                      uint32_t nlanes, const uint8_t *__restrict__ destuffed,
                                                      const RjTableSet *__restrict__ tabsets, RjCoefBuf coefs,
                                                      uint32_t epoch) {
  static_assert(RJ_WG == RJ_K1_WG, "lane layout granule");
#ifdef RJ_K1_PRIO
  __builtin_amdgcn_s_setprio(RJ_K1_PRIO);  // experiment: the serial chains win issue over co-resident K2 waves
#endif
  // lane-interleaved (LRow): 33 ring words per lane (the exact decoder's 32-word ring + mirror;
  // the chunk decoder uses 24) and RJ_STAGE staged entries per lane
  __shared__ __attribute__((aligned(16))) uint32_t s_ring[RJ_XRING_WORDS + 1][RJ_WG];
  __shared__ __attribute__((aligned(16))) uint32_t s_stage[RJ_STAGE][RJ_WG];
  __shared__ __attribute__((aligned(16))) uint16_t s_lut[RJ_SLUT_ENTRIES];
  __shared__ uint32_t s_T, s_ne;
  const uint32_t tid = threadIdx.x;
  if (tid == 0) s_ne = 0;
  const uint32_t g = lane0 + blockIdx.x * RJ_WG + tid;  // lane (kFallback: interval)
  bool pending = g < lane0 + nlanes;
  int i = 0;
  uint32_t gseg = 0, c = 0, nch = 1;
  if (pending) {
    gseg = kFallback ? g : rj_lane_seg(coefs, g);
    pending = kFallback ? gp(coefs.fallback)[g] != 0 : gseg != 0xFFFFFFFFu;
  }
  if (pending) {
    i = upper_index(nimg, gseg, [&](int q) { return imgs[q].seg_prefix; });
    if (!kFallback) {
      nch = rj_nch(coefs, gp(imgs[i].segs)[gseg - imgs[i].seg_prefix].src_len);
      c = nch - 1 - (g - rj_seg_lane0(coefs, gseg));  // reverse order: later chunks on earlier lanes
    }
  }
  const RjImageDev &im = imgs[i];
  const uint32_t seg = gseg - im.seg_prefix;
  const uint32_t my_ts = im.tabset;
  // one pass per distinct table set among the workgroup's lanes (normally exactly one)
  while (__syncthreads_or(pending)) {
    if (tid == 0) s_T = 0xFFFFFFFFu;
    __syncthreads();
    if (pending) atomicMin(&s_T, my_ts);
    __syncthreads();
    const uint32_t T = s_T;
    {
      const RjTableSet &ts = tabsets[T];
      uint4 *d4 = reinterpret_cast<uint4 *>(s_lut);
      constexpr uint32_t L1Q = RJ_LUT_L1 * 2 / 16, FQ = RJ_LUT_ENTRIES * 2 / 16;
      for (uint32_t q = tid; q < 2 * L1Q + 2 * FQ; q += RJ_WG) {
        const uint4 *s4;
        if (q < L1Q) s4 = reinterpret_cast<const uint4 *>(ts.dc[0].lut) + q;
        else if (q < 2 * L1Q) s4 = reinterpret_cast<const uint4 *>(ts.dc[1].lut) + (q - L1Q);
        else if (q < 2 * L1Q + FQ) s4 = reinterpret_cast<const uint4 *>(ts.ac[0].lut) + (q - 2 * L1Q);
        else s4 = reinterpret_cast<const uint4 *>(ts.ac[1].lut) + (q - 2 * L1Q - FQ);
        d4[q] = *gp(s4);
      }
    }
    __syncthreads();
    if (pending && my_ts == T) {
      pending = false;
      const RjSegDev sg = gp(im.segs)[seg];
      const uint32_t nblk = im.nblk_mcu;
      // per block-in-MCU b: component (2 bits) | dc table (1) | ac table (1), 4 bits each
      uint64_t binfo = 0;
      for (uint32_t b = 0; b < nblk; b++) {
        const uint32_t cc = im.blk_comp[b] & 3;
        binfo |= uint64_t(cc | ((im.comp_td[cc] & 1) << 2) | ((im.comp_ta[cc] & 1) << 3)) << (4 * b);
      }
      const uint32_t nbytes = sg.dst_len;
      const uint32_t blocks = sg.mcu_count * nblk;
      const uint8_t *data = destuffed + im.destuff_off + sg.dst_off;
      uint32_t *ent_base = coefs.ent + im.ent_off + sg.ent_off;
      const uint64_t ent_abs = im.ent_off + sg.ent_off;
      const uint32_t lane_first = rj_seg_lane0(coefs, gseg);
      const RjTableSet *ts = tabsets + T;
      LaneJob J;
      J.nbits = nbytes * 8u;
      J.blocks = blocks;
      J.missing = (sg.flags & RJ_SEG_MISSING) != 0;
      if (kFallback || nch == 1) {
        J.src = reinterpret_cast<const uint4 *>(data);
        J.bytes = nbytes;
        J.start_bit = 0;
        J.ent = ent_base;
        J.pieces = coefs.piece + lane_first;
        J.slots = rj_nch(coefs, sg.src_len);  // the interval's lanes: piece slots
        J.ent_abs = ent_abs;
        J.mcux = im.mcux;
        J.mcu_first = sg.mcu_first;
        J.mcu_count = sg.mcu_count;
        *gp(J.pieces) = RjPiece{ent_abs, 0u, blocks, 1u, {0, 0, 0}};
        const uint32_t ne = decode_exact<kFallback>(J, binfo, nblk, s_lut, ts, LRow{&s_ring[0][tid]},
                                                    LRow{&s_stage[0][tid]});
        if (coefs.count) atomicAdd(&s_ne, ne);
      } else {
        const uint32_t clen = rj_chunk_len(nbytes, nch);
        const uint32_t b0 = min(c * clen, nbytes), b1 = min(b0 + clen, nbytes);
        if (c > 0 && b0 >= nbytes) {  // no data left for this chunk (16-B rounding): nothing to decode
          RjChunkRes o = {};
          o.status = RJ_CHUNK_DONE;
          o.rb_over = 0xFFFFFFFFu;
          *gp(coefs.res + g) = o;
          put_record<kScope>(coefs.rec + uint64_t(g) * RJ_MAX_RECORDS, 0xFFFFFFFFu, 0u, epoch, 0u, 0u, 0, 0, 0);
          continue;
        }
        J.src = reinterpret_cast<const uint4 *>(data + b0);
        J.bytes = nbytes - b0;
        J.start_bit = b0 * 8u;
        J.end_bit = b1 * 8u;
        J.clen_bits = clen * 8u;
        J.ov_bit = J.end_bit + rj_chunk_reach(clen) * 8u;
        const uint32_t rcap = uint32_t(rj_chunk_cap(rj_chunk_len(sg.src_len, nch)));
        J.ent = coefs.ent + gp(coefs.seg_ent)[gseg] + uint64_t(c) * rcap;
        J.cap = rcap;
        J.spec = c > 0;
        J.rec = coefs.rec + uint64_t(g) * RJ_MAX_RECORDS;
        J.rec_next = J.rec - RJ_MAX_RECORDS;  // chunk c+1 sits on lane g-1
        J.next_chunks = nch - 1 - c;
        const uint32_t ne = decode_lane<true, kScope>(J, binfo, nblk, epoch, s_lut, ts, LRow{&s_ring[0][tid]},
                                                      LRow{&s_stage[0][tid]}, coefs.res + g);
        if (coefs.count) atomicAdd(&s_ne, ne);
      }
    }
  }
  // the loop exits through a barrier: every lane's count is in s_ne
  if (tid == 0 && coefs.count != nullptr && s_ne != 0) atomicAdd(coefs.count, (unsigned long long)s_ne);
}

// Chains the chunks of every split interval into pieces; flags intervals for the serial path.
__global__ __launch_bounds__(256) void k_resolve(const RjImageDev *__restrict__ imgs, int nimg, uint32_t nseg,
                                                 RjCoefBuf coefs) {
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  if (g >= nseg) return;
  const int i = upper_index(nimg, g, [&](int q) { return imgs[q].seg_prefix; });
  const RjImageDev &im = imgs[i];
  const RjSegDev sg = gp(im.segs)[g - im.seg_prefix];
  const uint32_t nch = rj_nch(coefs, sg.src_len);
  bool ok = true;
  if (nch > 1) {
    const uint32_t total = sg.mcu_count * im.nblk_mcu;
    // lane of chunk c under phase hypothesis h: lane_first + rj_chunk_lane(nch, hyp, c, h)
    const uint32_t lane_first = rj_seg_lane0(coefs, g), H = coefs.hyp;
    const uint64_t rcap = rj_chunk_cap(rj_chunk_len(sg.src_len, nch));
    const uint64_t ent0 = gp(coefs.seg_ent)[g];  // the call's chunk regions of this interval (one per lane)
    RjPiece *pieces = coefs.piece + lane_first;
    uint32_t c = 0, h = 0, vs_rb = 0, vs_ne = 0, T = 0, np = 0;
    int32_t D[3] = {0, 0, 0};
    while (true) {
      const uint32_t o = rj_chunk_lane(nch, H, c, h);
      const RjChunkRes r = gp(coefs.res)[lane_first + o];
      if (r.status != RJ_CHUNK_SYNC && r.status != RJ_CHUNK_DONE) { ok = false; break; }
      if (r.rb < vs_rb) { ok = false; break; }
      uint32_t nb = r.rb - vs_rb;
      if (r.status == RJ_CHUNK_DONE) {
        // a block the interval needs read past the data, or the data ended early: libjpeg's
        // insufficient-data semantics need the serial decode
        if (r.rb_over != 0xFFFFFFFFu && r.rb_over >= vs_rb && T + (r.rb_over - vs_rb) < total) { ok = false; break; }
        if (T + nb < total) { ok = false; break; }
      }
      if (T + nb > total) nb = total - T;
      gp(pieces)[np] = RjPiece{ent0 + uint64_t(o) * rcap + vs_ne, T, nb, 0u, {D[0], D[1], D[2]}};
      np++;
      T += nb;
      if (r.status == RJ_CHUNK_DONE || T >= total) break;
      const uint32_t t = c + (r.tgt & 0xFFFFu), th = r.tgt >> 16;
      if (t >= nch || t <= c || th >= H || r.rec >= RJ_MAX_RECORDS || np >= nch) { ok = false; break; }
      const RjRecord rec = gp(coefs.rec)[uint64_t(lane_first + rj_chunk_lane(nch, H, t, th)) * RJ_MAX_RECORDS + r.rec];
      for (int q = 0; q < 3; q++) D[q] = r.pred[q] + D[q] - rec.pred[q];
      c = t;
      h = th;
      vs_rb = rec.rb;
      vs_ne = rec.ne;
    }
    if (ok && T == total) gp(pieces)->npieces = np;
    else ok = false;
  }
  gp(coefs.fallback)[g] = ok ? 0u : 1u;
}

hipError_t LaunchEntropy(hipStream_t st, int stage, const RjImageDev *imgs, int nimg, uint32_t lanes_wg,
                         uint32_t lanes_dev, uint32_t nseg, const uint8_t *destuffed, const RjTableSet *tabsets,
                         RjCoefBuf coefs, uint32_t epoch) {
  if (nseg == 0) return hipSuccess;
  if (stage == 0) {
    if (lanes_wg)
      hipLaunchKernelGGL((k_entropy<false, __HIP_MEMORY_SCOPE_WORKGROUP>), dim3((lanes_wg + RJ_WG - 1) / RJ_WG),
                         dim3(RJ_WG), 0, st, imgs, nimg, 0u, lanes_wg, destuffed, tabsets, coefs, epoch);
    if (lanes_dev)
      hipLaunchKernelGGL((k_entropy<false, __HIP_MEMORY_SCOPE_AGENT>), dim3((lanes_dev + RJ_WG - 1) / RJ_WG),
                         dim3(RJ_WG), 0, st, imgs, nimg, lanes_wg, lanes_dev, destuffed, tabsets, coefs,
                         epoch);
  } else if (stage == 1) {
    hipLaunchKernelGGL(k_resolve, dim3((nseg + 255) / 256), dim3(256), 0, st, imgs, nimg, nseg, coefs);
  } else {
    hipLaunchKernelGGL((k_entropy<true, __HIP_MEMORY_SCOPE_WORKGROUP>), dim3((nseg + RJ_WG - 1) / RJ_WG),
                       dim3(RJ_WG), 0, st, imgs, nimg, 0u, nseg, destuffed, tabsets, coefs, epoch);
  }
  return hipGetLastError();
}

hipError_t LaunchEntropyLanes(hipStream_t st, const RjImageDev *imgs, int nimg, uint32_t lane0, uint32_t nlanes,
                              const uint8_t *destuffed, const RjTableSet *tabsets, RjCoefBuf coefs, uint32_t epoch) {
  if (nlanes == 0) return hipSuccess;
  hipLaunchKernelGGL((k_entropy<false, __HIP_MEMORY_SCOPE_WORKGROUP>), dim3((nlanes + RJ_WG - 1) / RJ_WG), dim3(RJ_WG),
                     0, st, imgs, nimg, lane0, nlanes, destuffed, tabsets, coefs, epoch);
  return hipGetLastError();
}

}  // namespace rj
