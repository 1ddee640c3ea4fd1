// rj_device.h -- descriptors shared by the host planner (rj_decoder.cpp) and the HIP kernels
// (rj_kernels.hip).  Plain PODs; every pointer is a device pointer on the handle's GPU.
//
// HBM layout of one batch (all regions carved from the handle's arena, rj_decoder.cpp):
//   images[]   RjImageDev          one per image in the batch
//   tabsets[]  RjTableSet          de-duplicated Huffman LUTs + natural-order quant tables
//   segs       RjSegDev per image  restart intervals (resident with the stream's ECS bytes)
//   destuffed  u8                  byte-unstuffed entropy data, each interval 16-B aligned
//   entries    uint32              sparse coefficients (K1 -> K2): per K1 chunk one stream,
//                                  per block its DC entry (zigzag pos 0) then its nonzero AC
//                                  entries, a terminator (pos 127) at the end; regions sized
//                                  for the worst case, 64-B aligned (RjCoefBuf)
//   pieces     RjPiece per chunk   which part of which stream holds which blocks
//   planes     u8                  per component, padded to the MCU grid (general path only)
#pragma once
#include <hip/hip_runtime.h>  // uint2/uint4 vector types (all users are built with hipcc)
#include <stdint.h>

#define RJ_MAX_BLK_MCU 10

// k_fused strips: one 64-lane workgroup per strip of S MCUs of one MCU row, at most one block
// per lane and at most RJ_FUSED_MAX_PX pixels wide (4:2:0 -> 10 MCUs = 160 px, 60 blocks).
#define RJ_FUSED_MAX_BLK 64
#define RJ_FUSED_MAX_PX 512
__host__ __device__ inline uint32_t rj_fused_strip_mcus(uint32_t hmax, uint32_t nblk_mcu) {
  const uint32_t a = RJ_FUSED_MAX_PX / (8u * hmax), b = RJ_FUSED_MAX_BLK / nblk_mcu;
  return a < b ? a : b;
}

// Sparse coefficient storage written by K1 and read by K2 (rj_fused.hip).
//   entry = uint16 value | zigzag position << 16 (positions 0..63; RJ_ENT_TERM ends a stream)
// K1 decodes every restart interval in one or more chunks (one lane each, see rj_entropy.hip);
// each chunk writes its own entry stream.  The pieces say which part of which stream is valid:
// piece j of an interval covers `nblk` blocks starting at the interval's block `first_blk`,
// read from entry `ent` (absolute index into `ent`) with `dcd` added to its DC values.
struct RjPiece {
  uint64_t ent;
  uint32_t first_blk, nblk;
  uint32_t npieces;  // in the interval's first piece; in a later piece of a lean split interval:
                     // the blocks of the stream at `ent` that precede the piece (its skip)
  int32_t dcd[3];
};
// chunk-start record (speculative lanes): block start at bit `pos` of the interval, block
// within the MCU in tag bits 0..3, call epoch in tag bits 4..31 (records persist across calls)
struct RjRecord {
  uint32_t pos, tag, ne, rb;  // ne: entries written before this block, rb: blocks before it
  int32_t pred[3];
  uint32_t pad;
};
// what a chunk's lane found when it stopped
struct RjChunkRes {
  uint32_t status;           // RJ_CHUNK_*
  uint32_t tgt, rec;         // SYNC: later chunk (chunks ahead, bits [15:0]; its hypothesis, [31:16]) and its record index
  uint32_t rb, ne;           // blocks / entries this lane produced before the stop point
  int32_t pred[3];           // its (chunk-relative) DC predictors at the stop point
  uint32_t rb_over;          // first block that read past the data (UINT32_MAX: none)
  uint32_t pad[3];
};
#define RJ_CHUNK_SYNC 1u      // reached a block start recorded by a later chunk with equal state
#define RJ_CHUNK_DONE 2u      // reached the end of the interval's data
#define RJ_CHUNK_FAIL 3u      // overlap or capacity exhausted: interval re-decoded serially
// K1 lanes: one per chunk, laid out per call by the host so that an interval of at most RJ_K1_WG
// chunks never straddles a workgroup (its lanes exchange chunk-start records through the CU's
// caches); longer intervals go to a second lane space whose records are exchanged device-wide.
// Within an interval the chunks run in reverse lane order (chunk c at lane seg_lane0 + nch-1-c).
#define RJ_K1_WG 256
struct RjCoefBuf {
  uint32_t *ent;              // entry streams
  RjPiece *piece;             // per lane; the interval's pieces start at its seg_lane0
  RjRecord *rec;              // per lane: RJ_MAX_RECORDS records
  RjChunkRes *res;            // per lane
  uint32_t *fallback;         // per interval (batch index): 1 = decode serially
  const uint32_t *lane_seg;   // per lane: batch interval index (0xFFFFFFFF: padding); null: identity
  const uint32_t *seg_lane0;  // per interval: its first lane; null: identity (no interval split)
  unsigned long long *count;  // profiling: entries written, summed per workgroup (null: off)
  const uint32_t *dense;      // progressive images: dense coefficients (RjImageDev.coef_off)
  uint32_t *wide_flag;        // host-mapped: set by K2 when it recorded a row for the fix-up
  uint32_t piece_shift;       // identity layout: interval s's pieces start at s << piece_shift
  uint32_t chunk_bytes;       // the call's chunk length (rj_chunks_cb; 0: no interval split)
  uint32_t warm_shift;        // k_huff_chunk warm-up: min(RJ_CHUNK_WARM_BYTES, chunk length >> warm_shift)
  const unsigned long long *seg_ent;  // per interval: first entry of its chunk regions (split ones)
  uint32_t hyp;               // MCU-phase hypotheses per speculative chunk (rj_chunk_lanes; 1: one lane per chunk)
  uint32_t wide_cap;          // K2: slots of the launch's fix-up list (the launches sharing one decode disjoint rows)
};
// Lean K1 split launch (rj_huff.hip): an interval decoded by a head lane from its start and a
// tail lane from rj_split_byte(dst_len); lane_seg entries carry the role in their top bits.
#define RJ_LANE_HEAD 0x40000000u
#define RJ_LANE_TAIL 0x80000000u
#define RJ_HL_SPLIT_DEC 256          // decoder lanes per workgroup of the split launch (two workgroups per CU)
#define RJ_HL_DEC5 320               // decoder lanes per workgroup of the five-wave lean launch
#define RJ_SPLIT_MIN_BYTES 1024u     // shorter intervals stay whole
__host__ __device__ inline uint32_t rj_split_byte(uint32_t dst_len) { return (dst_len * 29u / 64u) & ~15u; }
struct RjHuffSplit {
  uint64_t ent;  // first entry of the tail lanes' regions (pair p at ent + p * cap)
  uint64_t cap;  // entries per tail region
};
// K1 -> K2 hand-off inside one call (the "live" rows, rj_huff.hip hl_publish -> rj_fused.hip
// k_rows_live): a lean five-wave K1 decoder wave that has written its intervals' entries and
// pieces publishes those MCU rows (row images, one interval per row) into `slot`; K2 workgroups
// on a second stream take tickets in publication order and decode each row as soon as it is
// published, on the CUs whose K1 workgroup has finished.  A stream-ordered K2 after both takes
// the rows no ticket reached (k_rows_rest).
struct RjLive {
  unsigned long long *slot;  // per published row: epoch | (image << 11 | MCU row) << 32 (8-B sc1 granule)
  uint32_t *ctr;             // RJ_LIVE_* counters, zeroed per call in upload A
  uint32_t *cu_busy;         // per CU (rj_live_cu_key): K1 workgroups running there (zeroed in upload A)
  uint32_t epoch;            // this call's tag (never 0)
  uint32_t k1_groups;        // K1 workgroups (all must be resident before any K2 waits on a row)
  uint32_t k1_waves;         // K1 decoder waves (each reports once when it is done)
  uint32_t rows;             // rows the K1 launch may publish (the K2 grid)
};
#define RJ_LIVE_RESERVED 0  // slots reserved by K1 (published rows, once K1 is done)
#define RJ_LIVE_TICKET 1    // tickets taken by k_rows_live
#define RJ_LIVE_STARTED 2   // K1 workgroups started
#define RJ_LIVE_DONE 3      // K1 decoder waves done
#define RJ_LIVE_ERROR 4     // a ticket holder gave up on its row (never expected)
#define RJ_LIVE_GIVEUP 5    // K1 was not resident in time: the live launch leaves everything to k_rows_rest
#define RJ_LIVE_FINAL 6     // tickets taken before K1's last wave closed the counter
#define RJ_LIVE_CLOSED 0x80000000u  // RJ_LIVE_TICKET: no ticket is valid any more
#define RJ_LIVE_CTRS 16     // counter words (64 B)
#define RJ_LIVE_ROW_BITS 11 // MCU rows per image < 2^11 (16384 / 8)
#define RJ_LIVE_CU_KEYS 2048  // XCC (4 bits of HW_REG_XCC_ID) x CU / SH / SE (bits 8..15 of HW_REG_HW_ID)
// the CU this wave runs on, as an index below RJ_LIVE_CU_KEYS
__device__ __forceinline__ uint32_t rj_live_cu_key() {
#ifdef __HIP_DEVICE_COMPILE__
  const uint32_t hw = __builtin_amdgcn_s_getreg((7 << 11) | (8 << 6) | 4);   // hwreg(HW_REG_HW_ID, 8, 8)
  const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // hwreg(HW_REG_XCC_ID, 0, 4)
  return ((xcc & 7u) << 8) | (hw & 255u);
#else
  return 0;
#endif
}
#define RJ_ENT_PER_BLOCK 64       // worst case: DC + 63 AC (each position written at most once)
#define RJ_ENT_GROUP 16           // K1 writes entries in 64-B groups; regions are group-aligned
#define RJ_ENT_TERM (127u << 16)  // end-of-stream marker
#define RJ_ENT_SLACK 1024         // entries of read slack after the last region (K2 reads 512-entry windows)
#define RJ_MAX_RECORDS 64         // chunk-start records per speculative chunk
#define RJ_MAX_HYP 6              // MCU-phase hypotheses per speculative chunk at most (4:2:0's 6 blocks)
#ifndef RJ_RECORD_EVERY
#define RJ_RECORD_EVERY 8         // one record every 8th block start of a chunk's head
#endif

// Chunking of an interval of `bytes` raw entropy-coded bytes is decided per call
// (rj_decoder.cpp): the chunk length `cb` is the call's baseline bytes over one round of the
// chip's K1 decoder lanes (one k_huff_chunk workgroup of RJ_K1_WG lanes per CU), never below
// the handle's minimum; an interval of at least two chunk lengths is cut into floor(bytes / cb)
// chunks, one lane each, shorter ones are decoded whole by one lane with the exact serial
// semantics (so a large batch of MCU-row intervals keeps the lean K1).  A fixed 5 KB measured
// best on a 1024-image restart-less 1080p batch (c2nori, same box: 3 KB 150k, 4 KB 140k, 5 KB
// 178k, 5.5 KB 171k, 6 KB 168k, 7 KB 155k, 8 KB 149k images/s,
// profiles/r4_experiments/k1_chunk_bytes_ab.txt) -- exactly the length that fills one round --
// and small calls want short chunks (their lanes would leave the chip idle).  The
// resynchronisation costs ~1,000 bits per chunk boundary.
// RJ_CHUNK_BYTES: the parse-time default geometry (RjSegDev.chunk0, introspection only).
#ifndef RJ_CHUNK_BYTES
#define RJ_CHUNK_BYTES 5120u
#endif
#define RJ_CHUNK_MIN_BYTES 384u  // default floor of the call's chunk length (env RJ_CHUNK_MIN; sweep:
                                 // profiles/r4_experiments/call_shape_chunking.txt)
#define RJ_SPLIT_BYTES 12288u
#define RJ_OVERLAP_CHUNKS 3u      // a lane may decode this many chunk lengths past its own end,
#define RJ_OVERLAP_MIN_BYTES 4096u  // and at least this many bytes (resynchronisation is long-tailed)
#ifndef RJ_CHUNK_WARM_BYTES
#define RJ_CHUNK_WARM_BYTES 512u  // k_huff_chunk: the most a speculative lane starts before its chunk (16-B multiple)
#endif
#define RJ_CHUNK_ENT_PER_BYTE 4u  // region budget of a chunk lane (typical ~1.7); overflow -> serial path
__host__ __device__ inline uint32_t rj_chunks(uint32_t bytes) {
  if (bytes < RJ_SPLIT_BYTES) return 1u;
  const uint32_t n = (bytes + RJ_CHUNK_BYTES / 2) / RJ_CHUNK_BYTES;
  return n < 2 ? 1u : (n > 4096 ? 4096u : n);
}
// chunks of an interval under a call's chunk length cb (0: never split)
__host__ __device__ inline uint32_t rj_chunks_cb(uint32_t bytes, uint32_t cb) {
  if (cb == 0 || uint64_t(bytes) < 2ull * cb) return 1u;
  const uint32_t n = bytes / cb;
  return n > 4096 ? 4096u : n;
}
__host__ __device__ inline uint32_t rj_nch(const RjCoefBuf &c, uint32_t src_len) {
  return rj_chunks_cb(src_len, c.chunk_bytes);
}
// Lanes of an interval cut into nch chunks when each speculative chunk (c > 0) is decoded under
// `hyp` hypotheses of the MCU phase at its start (hypothesis h assumes block h of an MCU begins
// there): chunk 0 has one lane, every other chunk `hyp`.  A speculative decode that starts in the
// wrong phase keeps decoding a chroma block with the luma tables (or the reverse) until it slips
// into step by chance, which makes the resynchronisation long-tailed; one of the hypotheses starts
// in step and meets the true decode as soon as the symbols align.  Small calls, whose lanes leave
// the chip idle, take hyp = the MCU's block count (rj_decoder.cpp); large ones keep 1.
// Lane offsets inside the interval, reverse chunk order: chunk nch-1's hypotheses at [0, hyp), ...,
// chunk 1's at [(nch-2) hyp, (nch-1) hyp), chunk 0 at (nch-1) hyp.
__host__ __device__ inline uint32_t rj_chunk_lanes(uint32_t nch, uint32_t hyp) { return nch > 1 ? 1u + (nch - 1) * hyp : 1u; }
__host__ __device__ inline uint32_t rj_chunk_lane(uint32_t nch, uint32_t hyp, uint32_t c, uint32_t h) {
  return c == 0 ? (nch - 1) * hyp : (nch - 1 - c) * hyp + h;
}
// chunk length in bytes (16-B multiple); chunk c covers [c*len, min((c+1)*len, bytes))
__host__ __device__ inline uint32_t rj_chunk_len(uint32_t bytes, uint32_t nch) {
  return ((bytes + nch - 1) / nch + 15u) & ~15u;
}
__host__ __device__ inline uint64_t rj_group(uint64_t n) { return (n + RJ_ENT_GROUP - 1) / RJ_ENT_GROUP * RJ_ENT_GROUP; }
// entry region of one chunk of a split interval: a lane decodes at most its chunk +
// rj_chunk_reach more bytes; it stops (and the interval goes to the serial path, into its own
// region) before it would overflow.
__host__ __device__ inline uint32_t rj_chunk_reach(uint32_t clen) {
  return RJ_OVERLAP_CHUNKS * clen > RJ_OVERLAP_MIN_BYTES ? RJ_OVERLAP_CHUNKS * clen : RJ_OVERLAP_MIN_BYTES;
}
__host__ __device__ inline uint64_t rj_chunk_cap(uint32_t clen) {
  return rj_group(uint64_t(RJ_CHUNK_ENT_PER_BYTE) * (uint64_t(clen) + RJ_CHUNK_WARM_BYTES + rj_chunk_reach(clen)) +
                  2 * RJ_ENT_PER_BLOCK);
}
// entries reserved for an interval at parse time: one serial stream (zero-bit decode of the
// last MCU after the data ends, then one zero DC entry per skipped block) -- an exact lane's
// output, or the serial re-decode of a split interval the resolution failed
#ifndef RJ_EXP_ENT_PER_BYTE
#define RJ_EXP_ENT_PER_BYTE 8ull  // (timing probes only: a smaller reservation is unsafe for arbitrary tables)
#endif
__host__ __device__ inline uint64_t rj_interval_entries(uint32_t bytes, uint64_t blocks, uint32_t nblk_mcu) {
  return rj_group(RJ_EXP_ENT_PER_BYTE * bytes + blocks + uint64_t(nblk_mcu) * RJ_ENT_PER_BLOCK + 1);
}
// the chunk regions of an interval a call cuts into nch chunks, one per lane (RjCoefBuf.seg_ent:
// placed by the call after the images' serial regions; lane offset o's region at o x cap)
__host__ __device__ inline uint64_t rj_chunk_regions(uint32_t bytes, uint32_t nch, uint32_t hyp) {
  return uint64_t(rj_chunk_lanes(nch, hyp)) * rj_chunk_cap(rj_chunk_len(bytes, nch));
}

// One restart interval of one image (host parser rj_stream.cpp builds these).
struct RjSegDev {
  uint32_t src_off;    // raw ECS byte offset of the interval's first data byte
  uint32_t src_len;    // raw bytes (RST markers and trailing fill FFs excluded)
  uint32_t dst_off;    // destuffed byte offset (16-B aligned), relative to image.destuff_off
  uint32_t mcu_first;  // first MCU of the interval
  uint32_t mcu_count;  // MCUs in the interval
  uint32_t flags;      // RJ_SEG_MISSING: marker not found -> interval decodes to zero blocks
  uint32_t ent_off;    // first entry of the interval's region(s), relative to image.ent_off
  uint32_t chunk0;     // image-relative chunk count before this interval (rj_chunks(src_len) each)
  uint32_t dst_len;    // destuffed bytes (src_len minus the stuffed 00 and fill FF bytes)
  uint32_t pad[3];
};

// K0 work unit: up to RJ_DS_BLOCK raw bytes of one interval.  The host parser knows where every
// stuffed byte is (its marker scan visits each FF), so each block's output offset is known up
// front and the blocks are independent.
#ifndef RJ_DS_BLOCK
#define RJ_DS_BLOCK 2048u
#endif
struct RjDsBlock {
  uint32_t src_off;   // ECS-relative raw offset
  uint32_t len;       // raw bytes
  uint32_t dst_off;   // output offset relative to image.destuff_off
  uint32_t zero_end;  // last block of its interval: zero the output up to here (0: not last)
};
#define RJ_SEG_MISSING 1u

// GPU marker scan (rj_scan.hip): one job per stream, the post-SOS bytes at arena + src_off
struct RjScanOut {
  uint32_t ecs_end, nds, flags, destuff_bytes;  // flags 1: a list overflowed (host scan instead)
  unsigned long long entries;
  uint32_t nchunks, pad;
};
struct RjScanJob {
  unsigned long long src_off;
  uint32_t avail, ri, total_mcus, nblk_mcu;
  uint32_t expected, rst_cap, oth_cap, drop_cap;
  uint32_t ds_cap, pad[3];
  uint8_t *ecs;                     // resident ECS buffer (avail + 32 B)
  RjSegDev *segs, *segs_copy;       // resident table, and the copy the host plan reads back
  RjDsBlock *ds, *ds_copy;
  uint32_t *rst, *oth, *drop;       // scratch position lists
  RjScanOut *out;
};

// Canonical Huffman decoder for one table (T.81 Annex C), laid out for the GPU.
//   lut[0..511]      first level, indexed by the next 9 bits:
//                      (code_len << 8) | symbol      for codes of <= 9 bits
//                      0x8000 | sub                  longer codes: second level `sub`
//                      0xFFFF                        second-level pool exhausted: canonical search
//                      0x1100 (len 17, symbol 0)     no code: libjpeg's "bad code" result
//   lut[512 + sub*128 + next 7 bits]  second level for codes of 10..16 bits (same encoding)
#define RJ_LUT_L1 512
#define RJ_L2_SUBTABLES 8
#define RJ_LUT_ENTRIES (RJ_LUT_L1 + RJ_L2_SUBTABLES * 128)
#define RJ_LUT_BAD 0x1100u
struct RjHuffDev {
  uint16_t lut[RJ_LUT_ENTRIES];
  uint32_t maxcode16[18];  // exclusive upper bound of length-l codes, left-justified to 16 bits
  int32_t valoff[18];      // symbol index = (code >> (16 - l)) + valoff[l]
  uint8_t vals[256];
};

struct RjTableSet {
  RjHuffDev dc[2];
  RjHuffDev ac[2];
  uint16_t qz[4][64];  // zigzag (DQT) order, as stored by the parser (rocjpeg_parser.cpp:239)
};

// ---- lean K1 (rj_huff.hip): "row" images, whose every restart interval lies inside one MCU
// row, are decoded into raw entries and K2 restores the DC predictions ----
// One 32-bit table entry per code prefix; every field the symbol step needs is in it, for the
// symbol the prefix starts with (high half) and, where the prefix also holds the whole code of
// the symbol after it, for that second symbol (low half: a two-symbol step, rj_huff.hip):
//   [20:16] n1 = code bits + extra bits   [24:21] s1 (extra bits)
//   [30:25] R1: zigzag run (DC 0; AC r; ZRL 15; EOB 63 -> k >= 64)
//   [31]    code longer than the first level: [7:0] = AC second-level subtable, 0xFF = search
//   [4:0]   n2    [8:5] s2    [14:9] R2    [15] the second symbol is present
// A second symbol (always an AC symbol) is recorded only after a DC difference, an AC
// coefficient or ZRL whose bits and the second code all lie inside the first-level key (for a
// DC table: read with the AC table of the components that use it, when that is one table); the
// step takes it when the first symbol leaves the block open (k + R1 + 1 < 64).  Whether a symbol writes an entry follows from the fields: a DC
// symbol (k == 0) always, an AC symbol when s != 0.
// First levels: DC 9 bits, AC 11 bits; AC codes of 12..16 bits: up to RJ_HL_SUBS subtables of
// 32 entries (the next 5 bits) per table.
#define RJ_HL_DC_BITS 9
#define RJ_HL_AC_BITS 11
#define RJ_HL_SUBS 8
#define RJ_HL_AC_WORDS ((1 << RJ_HL_AC_BITS) + RJ_HL_SUBS * 32)
#define RJ_HL_DC_WORDS (1 << RJ_HL_DC_BITS)
#define RJ_HL_ESC 0x80000000u
#define RJ_HL_PAIR 0x8000u
struct RjLeanTables {  // LDS image: AC0, AC1 (first level + subtables), DC0, DC1
  uint32_t ac[2][RJ_HL_AC_WORDS];
  uint32_t dc[2][RJ_HL_DC_WORDS];
};
// Lean entry (lean K1 -> K2): [15:0] the coefficient as int16 (libjpeg HUFF_EXTEND of the
// symbol's s extra bits, done by K1 off its bit-position chain; for position 0 the DC
// *difference*), [22:16] zigzag position (corrupt runs past 63 clamped to 63, as libjpeg's
// natural-order table does; 127 = end of stream), bit 23: zero block (libjpeg's
// insufficient-data / missing-marker blocks: every coefficient 0, DC absolute), whose value
// field holds -32768 -- the marker restore_dc reads (no real DC difference is: |diff| <= 32767).
#define RJ_RE_TERM (127u << 16)
#define RJ_RE_ZERO ((1u << 23) | 0x8000u)

// Output jobs of the general (two-stage) path: one per written channel.
enum RjJobKind : uint32_t {
  RJ_JOB_COPY = 0,      // CopyChannel: surface plane bytes, dst pitch bytes per row
  RJ_JOB_RGB = 1,       // interleaved RGB
  RJ_JOB_RGB_PLANE = 2, // one of R/G/B planes (chan_sel)
  RJ_JOB_Y = 3,         // luma samples (also YUYV luma extraction)
  RJ_JOB_CHROMA = 4,    // planar U or V extracted from the surface model
};

struct RjJobDev {
  uint32_t image;
  uint32_t kind;
  uint32_t chan_sel;     // which surface plane / which RGB component / U(1) or V(2)
  uint32_t rows;         // rows written
  uint32_t row_bytes;    // bytes written per row
  uint32_t dst_pitch;
  uint8_t *dst;
  int32_t src_row0;      // surface row of output row 0
  int32_t src_byte0;     // surface byte (or pixel) column of output byte 0
  uint32_t row_prefix;   // exclusive prefix of rows over jobs (grid mapping)
  uint32_t pad;
};

// ---- progressive (SOF2) images (rj_prog.hip) ----
// Coefficients are accumulated densely: per component an MCU-padded raster of blocks, each 64
// int16 in zigzag order (32 dwords).  DC is two's complement (libjpeg's DC refinement ORs bit Al
// into it); AC is sign-magnitude (bit 15 = negative), so that every AC successive-approximation
// update -- first-scan value, refinement correction bit, newly nonzero coefficient -- is an OR
// into a word that no other scan of the same dependency level touches (rj_stream.cpp levels).
// A per-block 64-bit mask of nonzero AC positions (component raster of the blocks the AC scans
// code, no MCU padding) feeds the refinement scans.  Refinement scans do not touch the dense
// coefficients while they decode: each writes per-unit records (AC: the positions whose
// magnitude gains bit Al, the new coefficients and their signs; DC: one bit per block) with
// plain stores, and k_prog_fold applies a level's records (and the new nonzero positions) to
// the dense coefficients before the next level.
enum RjProgKind : uint8_t { RJ_PK_DC_FIRST = 0, RJ_PK_DC_REFINE = 1, RJ_PK_AC_FIRST = 2, RJ_PK_AC_REFINE = 3 };
struct RjProgScanDev {
  uint8_t kind, ns, ss, se;  // RjProgKind; components in the scan; spectral band
  uint8_t al, level, pad0, pad1;
  uint8_t comp[3];           // frame component of each scan component
  uint8_t hs[3], vs[3];      // blocks per unit of each scan component (1 x 1 unless interleaved)
  uint8_t tsel[3];           // which of the lane's two LDS tables (DC first)
  uint16_t tab[2];           // RjImageDev.ptabs index of table 0 / 1 (0xFFFF: none)
  uint32_t units_x, units;   // units (MCUs if interleaved, else blocks) per row / in total
  uint32_t ri;               // units per restart interval (0: one interval)
  uint32_t ival0;            // index of the scan's first interval in the image's interval list
  uint32_t nblk;             // blocks per unit
  // AC refinement: its producers -- the latest earlier scan of each coefficient of its band (AC
  // first or refinement; their nonzero masks are this scan's input, and each waited for its own
  // producers, rj_prog_stream.cpp); 0xFF: more than 3 (the call then runs level by level)
  uint8_t nprod, prod[3];
};
#define RJ_PROG_DONE 0xFFFFFFFFu  // interval progress: finished
#define RJ_WAVE_FIRST_DONE 1u      // k_prog_wave flag: first scans decoded before the grid (no waits on them)
#define RJ_WAVE_TEST_GIVEUP 2u     // k_prog_wave flag (tests): every producer wait gives up after a few polls
#define RJ_FOLD_ALL 0xFFFFFFFFu   // k_prog_fold level: every level (after a pipelined launch)
// AC refinement record of one unit (block): 32 B, written once by the decoding lane
struct RjRefineRec {
  unsigned long long orm;    // positions whose magnitude gains bit Al (correction 1 or new)
  unsigned long long sgn;    // new coefficients that are negative
  unsigned long long newm;   // new nonzero positions
  unsigned long long pad;
};
struct RjProgIvalDev {       // one restart interval of one scan
  uint32_t dst_off, dst_len; // destuffed bytes, relative to RjImageDev.destuff_off
  uint32_t unit0, nunits;
  uint16_t scan, flags;      // flags: RJ_SEG_MISSING (no marker: the interval is skipped)
  uint32_t rec_off;          // refinement scans: first record word (u64) of the interval, image-relative
};

struct RjImageDev {
  uint32_t width, height;
  uint32_t mcux, mcuy;
  uint8_t ncomp, nblk_mcu, interleaved, css;
  uint8_t hmax, vmax, fmt, roi;
  uint8_t comp_h[4], comp_v[4];
  uint8_t comp_td[4], comp_ta[4], comp_tq[4];
  uint8_t blk_comp[RJ_MAX_BLK_MCU], blk_dx[RJ_MAX_BLK_MCU], blk_dy[RJ_MAX_BLK_MCU];
  uint8_t comp_blk0[4];  // first block of each component inside an MCU
  uint32_t tabset;
  // inputs
  const uint8_t *ecs;
  const RjSegDev *segs;
  const RjDsBlock *ds;   // K0 blocks of this image
  uint32_t ds_prefix;    // exclusive prefix of K0 blocks over the batch
  uint32_t nseg;
  uint32_t seg_prefix;   // exclusive prefix of segments over the batch
  uint64_t destuff_off;  // into the destuffed buffer
  uint64_t ent_off;      // in entries (sparse coefficients), group-aligned
  uint32_t ri_mcus;      // MCUs per restart interval (0: one interval)
  uint32_t dc_diff;      // 1: lean K1 raw entries (DC differences; K2 restores the predictions)
  uint32_t idct_thr;     // |coefficient| above which the int32 IDCT may differ: (2^14 - 1) / max quantiser
  uint32_t chunk_prefix; // exclusive prefix of K1 chunks over the batch (unpadded)
  // component planes (general path)
  uint64_t plane_off[4];
  uint32_t plane_pitch[4], plane_rows[4];
  // output window (ROI semantics of rocjpeg_decoder.cpp:124-141)
  int32_t out_w, out_h, top, left;
  uint8_t *dst[4];
  uint32_t dst_pitch[4];
  // progressive (SOF2) only
  const RjProgScanDev *pscans;
  const RjProgIvalDev *pivals;
  const RjHuffDev *ptabs;
  uint64_t coef_off;      // dwords into the dense coefficient buffer (32 per block)
  uint64_t nz_off;        // masks into the nonzero-mask buffer
  uint64_t prec_off;      // u64 words into the refinement-record buffer
  uint32_t npscans;
  uint32_t pival_prefix;  // exclusive prefix of progressive intervals over the batch
  uint32_t progressive;
  uint32_t cblk0[3], wblk[3];   // dense block raster of each component (MCU-padded width)
  uint32_t nzblk0[3], cwblk[3]; // nonzero-mask raster (blocks the AC scans code)
  uint32_t chblk[3];
};
// k_prog_fold work: every block of one component of one image (64-block chunks, one wave each)
struct RjFoldJob {
  uint32_t image, comp, nblocks, chunk0;  // chunk0: exclusive prefix of chunks over the launch
};
