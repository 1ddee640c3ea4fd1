// rj_fused.hip -- K2 fused output kernel: dequant + ISLOW IDCT + nearest chroma upsample +
// YUV->RGB (or planar layouts) straight from the coefficient blocks to the caller's buffers.
//
// One workgroup = ONE wavefront (64 lanes) per strip of S MCUs of one MCU row, at most one
// block per lane (rj_fused_strip_mcus: 4:2:0 -> 10 MCUs = 160 x 16 px, 60 blocks).  Single-wave
// workgroups need no cross-wave barriers, so the ~17 strips resident per CU run out of phase
// and one strip's coefficient fetch (A) hides behind the others' IDCT / colour work (B, C).
//   A  zero the strip's LDS blocks, then lane b expands block b's sparse coefficient list
//      (K1's {start,count} index + 16-B aligned entries) into its block; block stride padded
//      to 144 B so that the per-lane ds_read_b128 of phase B is bank-conflict free.
//   B  lane b: block b's 64 coefficients into VGPRs, dequant, full 2-D ISLOW IDCT in
//      registers, 8 x 8-byte rows into the strip's component sample tiles (aliasing A).
//   C  lane = 4 consecutive pixels: one ds_read_b32 of luma, one ds_read_u16 (4:2:0/4:2:2)
//      or b32 (4:4:4) per chroma plane, 4 x (4 fma + 3 v_cvt_pk_u8_f32) packed straight
//      into 3 dwords -> one 12-B store per lane.
// HBM traffic per strip = its sparse coefficients (~4 B per nonzero + 8 B per block) read once +
// its output bytes written once.
//
// Same integer IDCT (rj_math.h) and CSC arithmetic as the general path, so both paths are
// bit-identical; eligibility (no ROI, canonical sampling geometry, copy channels with
// pitch == width) is decided on the host (rj_decoder.cpp FusedEligible).
#include <hip/hip_runtime.h>

#include <cstdio>

#include "rj_device.h"
#include "rj_kernels.h"
#include "rj_math.h"

namespace rj {

#define RJ_BLK_STRIDE 144  // bytes per staged block in LDS (128 + 16 pad)
#ifndef RJ_K2_OCC
#define RJ_K2_OCC 4  // K2 waves per SIMD the register budget is set for (128 VGPRs)
#endif
#ifndef RJ_K2_SPLIT_OCC
#define RJ_K2_SPLIT_OCC 3  // the split-aware instance (lean split calls): 133 VGPRs, no spills
#endif
#ifndef RJ_K2_DENSE_OCC
#define RJ_K2_DENSE_OCC 3  // the progressive (dense, int32 IDCT) K2: 168 VGPRs, no spills
#endif

#ifdef RJ_EXP_STAMPS  // diagnostic build: cycles per K2 phase, summed over waves (rj_decoder.cpp prints)
__device__ unsigned long long rj_stamp[8];
#define RJ_STAMP(var) const uint64_t var = __builtin_amdgcn_s_memtime()
#define RJ_STAMP_ADD(slot, d) acc[slot] += (d)
#else
#define RJ_STAMP(var)
#define RJ_STAMP_ADD(slot, d)
#endif

// byte b of w as float: the backend selects v_cvt_f32_ubyte{0..3} for this pattern
__device__ __forceinline__ float u8f(uint32_t w, int b) { return float((w >> (8 * b)) & 255u); }

// 4 pixels -> 12 bytes RGB.  y4: 4 luma bytes; u/v: per-pixel chroma as float minus 128.
// Arithmetic and packing order exactly as rocjpeg_hip_kernels.cpp:1431-1443 / :25-30.
__device__ __forceinline__ void csc4(uint32_t y4, const float (&u)[4], const float (&v)[4], uint32_t &d0, uint32_t &d1,
                                     uint32_t &d2) {
  float r[4], g[4], b[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const float fy = u8f(y4, j);
    r[j] = fmaf(1.5748f, v[j], fy);
    g[j] = fmaf(-0.4681f, v[j], fmaf(-0.1873f, u[j], fy));
    b[j] = fmaf(1.8556f, u[j], fy);
  }
  d0 = __builtin_amdgcn_cvt_pk_u8_f32(r[1], 3, __builtin_amdgcn_cvt_pk_u8_f32(b[0], 2,
       __builtin_amdgcn_cvt_pk_u8_f32(g[0], 1, __builtin_amdgcn_cvt_pk_u8_f32(r[0], 0, 0u))));
  d1 = __builtin_amdgcn_cvt_pk_u8_f32(g[2], 3, __builtin_amdgcn_cvt_pk_u8_f32(r[2], 2,
       __builtin_amdgcn_cvt_pk_u8_f32(b[1], 1, __builtin_amdgcn_cvt_pk_u8_f32(g[1], 0, 0u))));
  d2 = __builtin_amdgcn_cvt_pk_u8_f32(b[3], 3, __builtin_amdgcn_cvt_pk_u8_f32(g[3], 2,
       __builtin_amdgcn_cvt_pk_u8_f32(r[3], 1, __builtin_amdgcn_cvt_pk_u8_f32(b[2], 0, 0u))));
}

// wave-uniform value: keeps it in an SGPR (the byte-sized descriptor fields arrive through
// vector loads, which would otherwise pin a VGPR copy per uniform value across the strip loop)
__device__ __forceinline__ uint32_t U(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ void store_bytes(uint8_t *d, uint32_t n, const uint32_t *w) {
#pragma unroll
  for (int j = 0; j < 12; j++)
    if (uint32_t(j) < n) gp(d)[j] = uint8_t(w[j >> 2] >> (8 * (j & 3)));
}

// Entry-stream window of one wave: w[r] = ent[base + r * 64 + lane] (coalesced rows).  The
// loads of the next strip's window are issued as soon as its start is known (end of phase A)
// and complete behind the IDCT and output phases.
#ifndef RJ_WIN_ROWS
#define RJ_WIN_ROWS 8
#endif
struct EntWin {
  uint32_t w[RJ_WIN_ROWS];
  uint32_t base_lo, base_hi;

  __device__ __forceinline__ void load(const uint32_t *__restrict__ ent, uint64_t at, uint32_t lane) {
    base_lo = U(uint32_t(at));
    base_hi = U(uint32_t(at >> 32));
    const uint32_t *p = ent + at;
#pragma unroll
    for (int r = 0; r < RJ_WIN_ROWS; r++) w[r] = gp(p)[r * 64u + lane];
  }
  // wait here for the window's loads.  vmcnt is in order on gfx9: a wait for a window row issued
  // after the previous strip's pixel stores waits for those stores too.  parse_blocks' walk over a
  // window has no waits when every path into it settled the window first: after each load inside
  // parse_blocks and the row's first, and in row_body after the IDCT for the next strip's window
  // (loaded at the end of phase A, waited before phase C's stores).
  __device__ __forceinline__ void settle() {
#pragma unroll
    for (int r = 0; r < RJ_WIN_ROWS; r++) asm volatile("" : "+v"(w[r]));
  }
};

// Position in the image's entry streams: the next block's DC entry inside the current piece
// (RjPiece: which part of which K1 chunk stream holds which blocks of an interval).
struct Nav {
  uint32_t cur_lo, cur_hi;  // absolute entry index (64-bit, kept as two SGPR-able halves)
  uint32_t bleft;           // blocks left in the current piece
  uint32_t seg, pj;         // interval (image-relative) and piece within it
  int32_t dcd[3];           // DC correction of the current piece, per component
  uint32_t skip;            // blocks at cur() to pass over before the piece (lean split tails)
  uint32_t term;            // 1: a lean split tail that may end before its blocks (terminator check)
  __device__ __forceinline__ uint64_t cur() const { return uint64_t(cur_hi) << 32 | cur_lo; }
  __device__ __forceinline__ void set_cur(uint64_t v) {
    cur_lo = U(uint32_t(v));
    cur_hi = U(uint32_t(v >> 32));
  }
  __device__ __forceinline__ void take(const RjPiece *pc) {
    const RjPiece p = *gp(pc);
    set_cur(p.ent);
    bleft = U(p.nblk);
    dcd[0] = int32_t(U(uint32_t(p.dcd[0])));
    dcd[1] = int32_t(U(uint32_t(p.dcd[1])));
    dcd[2] = int32_t(U(uint32_t(p.dcd[2])));
    skip = 0;
    term = 0;
  }
};
template <bool B>
struct BoolC {
  static constexpr bool value = B;
};

// Expand the next `nb` blocks of the entry streams into the zeroed LDS blocks [0, nb) (block j
// at s_buf + j * RJ_BLK_STRIDE, int16 in zigzag order), after discarding `drop` blocks.  A
// block starts at its DC entry (pos 0); a terminator (pos 127) ends a stream; a block has
// <= 64 entries.  Entries are consumed row by row from the window; the ordinal of an entry's
// block is the number of block starts at or before it, so rows need no alignment to blocks.
// cbits: component of each block within the MCU (2 bits each), for the DC corrections.
// Lane masks straight from v_cmp into an SGPR pair.  (A __ballot of an or of compares, or of a
// bool that is also used per lane, is re-materialised by the compiler as v_cndmask + v_cmp per
// row of the scatter.)  v_cmp writes 0 for inactive lanes, which is the ballot's meaning.
// ballot(p == 0 || p == 127): block starts and the terminator
__device__ __forceinline__ uint64_t mask_start(uint32_t p) {
  uint64_t a, b;
  asm volatile("v_cmp_eq_u32_e64 %0, 0, %2\n\tv_cmp_eq_u32_e64 %1, %3, %2\n\ts_or_b64 %0, %0, %1"
               : "=&s"(a), "=&s"(b)
               : "v"(p), "s"(127u));
  return a;
}


// kPairs (the main K2 instances): each coefficient is dequantised here and stored scaled into
// its block's pair layout (rj_math.h idct_dot2_block): entry value x quantiser (i24 multiply,
// exact for 16-bit quantisers) x 32, the DC x 16 (raw DC differences stay as they are: restore_dc
// finishes them).  A coefficient outside the dot2 IDCT's exact domain raises `bad` (the row goes
// to the fix-up launch).  The entry's block in the strip supplies, through one ds_bpermute of the
// owning lane's `lane_info` (block LDS base | 4 x component << 16), where the block lives and which
// component's quantisers apply; s_qw[3 p + c] = quantiser | pair-layout byte offset << 16.
// !kPairs (the fix-up instances): raw coefficients in zigzag order, checked against the int32
// IDCT's domain (thr, on the raw value) -- the layout idct_pass1_wide reads.
template <bool kRaw, bool kSplit, bool kPairs>
__device__ __forceinline__ void parse_blocks(const RjImageDev &im, const RjCoefBuf &coefs,
                                             const uint32_t *__restrict__ ent, uint32_t lane, uint32_t nb,
                                             uint32_t drop, uint32_t nblk, uint32_t cbits, EntWin &win, Nav &nv,
                                             uint8_t *s_buf, const uint32_t *s_qw, uint32_t lane_info, int thr,
                                             bool &bad) {
  uint32_t done = 0;
  const uint32_t need = nb + drop;
  uint32_t bad_l = 0;  // this lane stored a coefficient outside the IDCT's exact domain (one ballot at the end)
  for (uint32_t moves = 0; done < need && moves < (1u << 16); moves++) {  // bounded on corrupt pieces
    if (nv.bleft == 0) {  // next piece, or the first piece of the next interval (synchronous reload)
      if (nv.seg >= im.nseg) break;
      // U(): the slot load completes here, on every path (a load left in flight into the merge
      // below made the waitcnt pass put a vmcnt(0) in the scatter's window loop, which then also
      // waited for the previous strip's pixel stores)
      const RjPiece *pb = coefs.piece + U(rj_seg_lane0_k<kSplit>(coefs, im.seg_prefix + nv.seg));
      if (nv.pj + 1 < U(gp(pb)->npieces)) {
        nv.pj++;
      } else {
        nv.seg++;
        nv.pj = 0;
        if (nv.seg >= im.nseg) break;
        pb = coefs.piece + U(rj_seg_lane0_k<kSplit>(coefs, im.seg_prefix + nv.seg));
      }
      nv.take(pb + nv.pj);
      if (kRaw && kSplit && nv.pj > 0) {  // a split interval's tail: skip count, bit 31 may end early
        const uint32_t f = U(gp(pb + nv.pj)->npieces);
        nv.skip = f & 0x7FFFFFFFu;
        nv.term = f >> 31;
      }
      win.load(ent, nv.cur(), lane);
      win.settle();
    }
    // a split tail's piece starts after `skip` blocks of its stream: pass over them first
    const bool pass = kSplit && nv.skip != 0;
    const uint32_t piece = pass ? nv.skip : min(need - done, nv.bleft);  // blocks taken from this piece
    const bool fix_dc = !kRaw && (nv.dcd[0] | nv.dcd[1] | nv.dcd[2]) != 0;
    uint32_t seen = 0;                                  // block starts before the current row
    // entries stored: 0 <= rel < piece + done - drop (ord < piece, and not a dropped block), as
    // one unsigned compare of 4 rel
    const int32_t lim_s = int32_t(piece + done) - int32_t(drop);
    const uint32_t st_lim4 = (pass || lim_s < 0) ? 0u : uint32_t(lim_s) * 4u;
    const uint32_t end4 = uint32_t(lim_s) * 4u;  // rel4 of the block past the piece
    // one pass over the window in registers; true when the piece ends inside it
    // kT: the terminator check of a lean split tail that may end early (only those pay for it)
    auto walk = [&](auto kT) __attribute__((always_inline)) -> bool {
      constexpr bool kTerm = kRaw && kSplit && decltype(kT)::value;
#pragma unroll
      for (int r = 0; r < RJ_WIN_ROWS; r++) {
        const uint32_t e = win.w[r];
        // zigzag position at [22:16] (127: end of stream; lean K1 clamps corrupt runs to 63)
        const uint32_t p_raw = (e >> 16) & 127u;
        const uint32_t p = p_raw;
        const uint64_t m = mask_start(p_raw);  // block starts (and the terminator): p_raw 0 or 127
        // ord = block starts at or before this lane, - 1: the count of m's bits 1..lane (mbcnt of
        // m >> 1) plus bit 0, in scalar terms -- no per-lane copy of the start flag
        const uint64_t m1 = m >> 1;
        const uint32_t incl = __builtin_amdgcn_mbcnt_hi(uint32_t(m1 >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m1), 0u));
        const uint32_t ord0 = seen + uint32_t(m & 1u) - 1u;  // ord = incl + ord0
        const uint32_t ord = incl + ord0;
        // the entry's block in the strip (negative: a dropped block), and 4x it in one
        // v_lshl_add from the mbcnt: the bpermute address, the store bound and the piece end all
        // compare on rel4 (4 rel mod 2^32 -- |rel| < 2^30)
        const int32_t rel = int32_t(ord + (done - drop));
        const uint32_t rel4 = (incl << 2) + (ord0 + (done - drop)) * 4u;
        // a split interval's tail piece may end early (its lane stopped at libjpeg's
        // insufficient-data point): the piece's remaining blocks are zero blocks, and nothing
        // after its terminator belongs to the stream
        const uint64_t term = kTerm ? __ballot(p == 127 && ord < piece) : 0ull;
        const int tl = term ? __ffsll((long long)term) - 1 : 64;
        // the entry's block in the strip, and from its lane: LDS base, quantiser row (whole wave)
        // (ds_bpermute takes the source lane from address bits [7:2]: rel mod 64, no masking)
        const uint32_t info = kPairs ? uint32_t(__builtin_amdgcn_ds_bpermute(int(rel4), int(lane_info))) : 0u;
        if (rel4 < st_lim4 && p < 64u && (!kTerm || int(lane) < tl)) {
          int v = int(int16_t(e & 0xFFFFu));  // lean entries: K1 applied HUFF_EXTEND
          if constexpr (kPairs) {
            // component-interleaved s_qw[3 p + c]: (a/4) mod 32 banks; info >> 16 = 4 c (bytes)
            const uint32_t qe = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(s_qw) +
                                                                    __umul24(p, 12u) + (info >> 16));
            if (!kRaw && fix_dc && p == 0) {
              const uint32_t cc = info >> 18;
              v += cc == 0 ? nv.dcd[0] : (cc == 1 ? nv.dcd[1] : nv.dcd[2]);
            }
            // |v| < 2^15, q < 2^16: exact in the i24 multiply.  Raw entries: one SDWA multiply of
            // the entry's low half (sign-extended) by the quantiser (low half of qe)
            int x;
            if constexpr (kRaw)
              asm("v_mul_i32_i24_sdwa %0, sext(%1), %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0"
                  : "=v"(x) : "v"(e), "v"(qe));
            else
              x = __mul24(v, int(qe & 0xFFFFu));
            // straight-line selects (no divergent DC / AC branches in the scatter)
            const bool dc = p == 0;
            int sv;
            if constexpr (kRaw) {  // a raw DC is a difference (restore_dc finishes it)
              const bool oob = !dc && uint32_t(x + RJ_DOT2_AC_MAX) > uint32_t(2 * RJ_DOT2_AC_MAX);
              bad_l = oob ? 1u : bad_l;
              // the DC difference is the entry's low half (ds_write_b16); a zero block's is -32768
              sv = dc ? int(e) : x << 5;
            } else {
              const int lim = dc ? RJ_DOT2_DC_MAX : RJ_DOT2_AC_MAX;
              const bool oob = uint32_t(x + lim) > uint32_t(2 * lim);
              bad_l = oob ? 1u : bad_l;
              sv = x << (dc ? 4 : 5);
            }
            *reinterpret_cast<int16_t *>(s_buf + (info & 0xFFFFu) + (qe >> 16)) = int16_t(sv);
          } else {
            if (!kRaw && fix_dc && p == 0) {
              const uint32_t bi = uint32_t(rel) % nblk;  // strips start at an MCU boundary
              const uint32_t cc = (cbits >> (2 * bi)) & 3u;
              v += cc == 0 ? nv.dcd[0] : (cc == 1 ? nv.dcd[1] : nv.dcd[2]);
            }
            // outside the int32 IDCT's exact domain (raw DC: a difference, checked by restore_dc)
            const bool oob = (!kRaw || p != 0) && int16_t(v) != -32768 && abs(int(int16_t(v))) > thr;
            bad_l = oob ? 1u : bad_l;
            *reinterpret_cast<int16_t *>(s_buf + __umul24(uint32_t(rel), uint32_t(RJ_BLK_STRIDE)) + p * 2) = int16_t(v);
          }
        }
        if (term) {
          const uint32_t t_ord = pass ? piece : __builtin_amdgcn_readlane(ord, tl);
          for (uint32_t z = t_ord + lane; z < piece; z += 64)
            if (done + z >= drop) *reinterpret_cast<int16_t *>(s_buf + (done + z - drop) * RJ_BLK_STRIDE) = int16_t(-32768);
          nv.set_cur((uint64_t(win.base_hi) << 32 | win.base_lo) + uint32_t(r) * 64u + uint32_t(tl));
          return true;
        }
        const uint64_t hit = __ballot(rel4 == end4) & m;  // start of the first block past the piece (ord == piece)
        seen += __popcll(m);
        if (hit) {
          nv.set_cur((uint64_t(win.base_hi) << 32 | win.base_lo) + uint32_t(r) * 64u +
                     uint32_t(__ffsll((long long)hit) - 1));
          return true;
        }
      }
      return false;
    };
    bool found = false;
    for (uint32_t guard = 0; !found && guard < (1u << 20); guard++) {  // bounded even on a corrupt stream
      if (guard) {  // the next window, settled: walk() then has no waits on any path (see EntWin::settle)
        win.load(ent, (uint64_t(win.base_hi) << 32 | win.base_lo) + RJ_WIN_ROWS * 64u, lane);
        win.settle();
      }
      found = (kRaw && kSplit && nv.term) ? walk(BoolC<true>{}) : walk(BoolC<false>{});
    }
    if (pass) {
      nv.skip = 0;
      win.load(ent, nv.cur(), lane);  // the piece proper starts mid-window
      win.settle();
    } else {
      done += piece;
      nv.bleft -= piece;
    }
  }
  if (__ballot(bad_l != 0) != 0) bad = true;
}

// DC prediction of a strip of raw-entry blocks (lean K1 wrote differences; T.81 F.2.1.3.1):
// lane = block of the strip (MCU order), its component c.  Per component an inclusive scan of
// the differences over the strip, plus the running predictor `carry` of the previous strips of
// the row; a restart interval starting inside the strip (every ri MCUs) resets it there.  Zero
// blocks (marked -32768) are absolute 0 (libjpeg's insufficient data / missing marker: every
// later block of the interval is one too).  Writes the absolute DC back into the LDS block.
// kPairs: the DC is stored dequantised x 16 (q0: this lane's component's DC quantiser) and
// checked against the dot2 IDCT's domain; otherwise raw, checked against thr.
template <bool kPairs>
__device__ __forceinline__ bool restore_dc(uint8_t *s_buf, uint32_t tid, uint32_t nb, uint32_t nblk, uint32_t c,
                                           uint32_t mx0, uint32_t mcu_row0, uint32_t ri, int (&carry)[3], int thr,
                                           uint32_t q0) {
  int16_t *dcp = reinterpret_cast<int16_t *>(s_buf + tid * RJ_BLK_STRIDE);
  const int d = tid < nb ? int(*dcp) : 0;
  const bool zero = d == -32768;
  const int dd = zero ? 0 : d;
  // the last interval start at or before this block's MCU, as a lane (-1: before the strip)
  const uint32_t m = mcu_row0 + mx0 + tid / nblk;
  const uint32_t mstart = m - m % ri;
  const int rlane = mstart >= mcu_row0 + mx0 ? int((mstart - mcu_row0 - mx0) * nblk) : -1;
  int pred = 0;
  // an interval starting inside the strip past its first lane (a restart interval shorter than
  // the strip) needs the scan value in front of it; with row intervals none does
  const bool mid = __ballot(tid < nb && rlane > 0) != 0;
#pragma unroll
  for (uint32_t cc = 0; cc < 3; cc++) {
    const int sc = wave_scan(c == cc ? dd : 0);
    // value of the scan just before the reset lane (0 if the reset is at lane 0)
    const int before = mid ? __shfl(sc, rlane > 0 ? rlane - 1 : 0) : 0;
    const int mine = rlane < 0 ? carry[cc] + sc : sc - (rlane > 0 ? before : 0);
    if (c == cc) pred = mine;
    // the next strip starts from the last block's predictor
    const int last = __builtin_amdgcn_readlane(mine, int(nb - 1));
    carry[cc] = last;
  }
  const int16_t dc = int16_t(zero ? 0 : pred);  // libjpeg keeps the predictor wide, stores (JCOEF)
  if constexpr (kPairs) {
    const int x = __mul24(int(dc), int(q0));
    if (tid < nb) *dcp = int16_t(x << 4);
    return __ballot(tid < nb && uint32_t(x + RJ_DOT2_DC_MAX) > uint32_t(2 * RJ_DOT2_DC_MAX)) != 0;
  } else {
    if (tid < nb) *dcp = dc;
    return __ballot(tid < nb && abs(int(dc)) > thr) != 0;  // outside the int32 IDCT's exact domain
  }
}

// Two sign-magnitude int16 (bit 15 = negative) -> two's complement, per half (packed ops).
__device__ __forceinline__ uint32_t sm16x2_to_tc(uint32_t w) {
  typedef short s16x2 __attribute__((ext_vector_type(2)));
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  const s16x2 sx = __builtin_bit_cast(s16x2, w) >> 15;  // 0 or -1 per half
  const u16x2 x = __builtin_bit_cast(u16x2, (w & 0x7FFF7FFFu) ^ __builtin_bit_cast(uint32_t, sx));
  return __builtin_bit_cast(uint32_t, u16x2(x - __builtin_bit_cast(u16x2, sx)));
}

// Progressive images: this lane's block (component c, block column bx of the strip, row by) from
// the dense coefficients into its LDS slot, AC converted to two's complement (DC already is).
__device__ __forceinline__ void load_dense_block(const RjImageDev &im, const uint32_t *__restrict__ dense,
                                                 uint32_t lane_blk, uint32_t mx0, uint32_t my, bool inter,
                                                 uint8_t *slot) {
  const uint32_t c = lane_blk >> 12;
  const uint32_t hc = inter ? im.comp_h[c] : 1, vc = inter ? im.comp_v[c] : 1;
  const uint32_t bx = mx0 * hc + (lane_blk & 255u), by = my * vc + ((lane_blk >> 8) & 15u);
  const uint32_t cb = c == 0 ? im.cblk0[0] : (c == 1 ? im.cblk0[1] : im.cblk0[2]);
  const uint32_t wb = c == 0 ? im.wblk[0] : (c == 1 ? im.wblk[1] : im.wblk[2]);
  const uint4 *src = reinterpret_cast<const uint4 *>(dense + im.coef_off + uint64_t(cb + by * wb + bx) * 32u);
  uint4 v[8];
#pragma unroll
  for (int q = 0; q < 8; q++) v[q] = gp(src)[q];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    uint4 o;
    o.x = sm16x2_to_tc(v[q].x);
    if (q == 0) o.x = (o.x & 0xFFFF0000u) | (v[q].x & 0xFFFFu);  // DC: two's complement already
    o.y = sm16x2_to_tc(v[q].y);
    o.z = sm16x2_to_tc(v[q].z);
    o.w = sm16x2_to_tc(v[q].w);
    *reinterpret_cast<uint4 *>(slot + q * 16) = o;
  }
}

// K2: one wavefront per MCU row of one image, looping over the row's strips of S MCUs.
//   kPlanes = false: fused output (rj_decoder.cpp FusedEligible images)
//   kPlanes = true : general path, blocks into the MCU-padded component planes (K2b reads them)
//   kDense = true  : progressive images -- blocks come from the dense coefficient buffer
//                    (rj_prog.hip layout: zigzag, AC sign-magnitude) instead of entry streams
// (image i, MCU row my) of a K2 launch: from an explicit list, or from the per-image row prefix
__device__ __forceinline__ void row_of_block(const RjImageDev *__restrict__ imgs, int nimg,
                                             const uint32_t *__restrict__ row_prefix, const uint2 *__restrict__ row_list,
                                             uint32_t w, int &i, uint32_t &my) {
  if (row_list != nullptr) {  // pipelined launch: an explicit (image, row) list for this group
    const uint2 e = row_list[w];
    i = int(U(e.x));
    my = U(e.y);
  } else {
    // interpolation guess (exact for a batch of equal image heights: two independent loads),
    // then a binary search on the side it missed
    const uint32_t nrows = gridDim.x;
    int g = int(min(uint64_t(w) * uint64_t(nimg) / max(nrows, 1u), uint64_t(nimg - 1)));
    const uint32_t pg = row_prefix[g], pg1 = g + 1 < nimg ? row_prefix[g + 1] : 0xFFFFFFFFu;
    int lo = 0, hi = nimg - 1;
    if (pg <= w && w < pg1) lo = hi = g;
    else if (pg > w) hi = g - 1;
    else lo = g + 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (row_prefix[mid] <= w) lo = mid;
      else hi = mid - 1;
    }
    i = __builtin_amdgcn_readfirstlane(lo);  // wave-uniform: image fields become scalar loads
    my = w - row_prefix[i];
  }
}

// 4 pixels -> 12 bytes RGB with packed fp32 (v_pk_fma_f32: two fmas per instruction, each
// rounded exactly as v_fma_f32), pixels (0,1) and (2,3) in the two halves.  Same arithmetic and
// packing order as csc4.  u01 / v01: chroma (as float minus 128) of pixels 0..1 / 2..3 when
// they share it (kHs), else the per-pixel values are passed in pairs.
typedef float rj_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void csc4_pk(uint32_t y4, rj_f2 ua, rj_f2 ub, rj_f2 va, rj_f2 vb, uint32_t &d0,
                                        uint32_t &d1, uint32_t &d2) {
  const rj_f2 ya = {u8f(y4, 0), u8f(y4, 1)}, yb = {u8f(y4, 2), u8f(y4, 3)};
  const rj_f2 kr = {1.5748f, 1.5748f}, kgu = {-0.1873f, -0.1873f}, kgv = {-0.4681f, -0.4681f}, kb = {1.8556f, 1.8556f};
  const rj_f2 ra = __builtin_elementwise_fma(kr, va, ya), rb = __builtin_elementwise_fma(kr, vb, yb);
  const rj_f2 ga = __builtin_elementwise_fma(kgv, va, __builtin_elementwise_fma(kgu, ua, ya));
  const rj_f2 gb = __builtin_elementwise_fma(kgv, vb, __builtin_elementwise_fma(kgu, ub, yb));
  const rj_f2 ba = __builtin_elementwise_fma(kb, ua, ya), bb = __builtin_elementwise_fma(kb, ub, yb);
  d0 = __builtin_amdgcn_cvt_pk_u8_f32(ra.y, 3, __builtin_amdgcn_cvt_pk_u8_f32(ba.x, 2,
       __builtin_amdgcn_cvt_pk_u8_f32(ga.x, 1, __builtin_amdgcn_cvt_pk_u8_f32(ra.x, 0, 0u))));
  d1 = __builtin_amdgcn_cvt_pk_u8_f32(gb.x, 3, __builtin_amdgcn_cvt_pk_u8_f32(rb.x, 2,
       __builtin_amdgcn_cvt_pk_u8_f32(ba.y, 1, __builtin_amdgcn_cvt_pk_u8_f32(ga.y, 0, 0u))));
  d2 = __builtin_amdgcn_cvt_pk_u8_f32(bb.y, 3, __builtin_amdgcn_cvt_pk_u8_f32(gb.y, 2,
       __builtin_amdgcn_cvt_pk_u8_f32(rb.y, 1, __builtin_amdgcn_cvt_pk_u8_f32(bb.x, 0, 0u))));
}

// Phase C fast path: interleaved RGB of a 3-component image over a whole strip inside the
// image, 4-byte aligned destination -- no per-quad bounds and no format branches in the loop.
// Lane = 4 consecutive pixels of one row (12 output bytes, one dwordx3 store); kHs / kVs:
// chroma halved horizontally / vertically (4:2:0 both, 4:2:2 kHs, 4:4:4 neither).
// kVs: a lane takes the 4 x 2 pixels of two rows that share one chroma row (the chroma is read
// and converted once for both), so qy counts row pairs.
template <bool kHs, bool kVs>
__device__ __forceinline__ void rgb_strip(const uint8_t *ty, const uint8_t *tu, const uint8_t *tv, uint32_t tw0,
                                          uint32_t tw1, uint32_t tid, uint32_t quads_x, uint32_t rows, uint8_t *dst,
                                          uint32_t pitch) {
  const uint32_t qsy = 64 / quads_x, qsx = 64 - qsy * quads_x;
  uint32_t qy = tid / quads_x, qx = tid - qy * quads_x;
  const uint32_t nq = kVs ? rows >> 1 : rows;  // kVs: rows is even (an MCU row of 16)
  while (qy < nq) {
    const uint32_t x = qx * 4;
    const uint32_t yrow = kVs ? 2 * qy : qy;
    const uint32_t y4 = *reinterpret_cast<const uint32_t *>(ty + __umul24(yrow, tw0) + x);
    const uint32_t crow = __umul24(qy, tw1);
    const rj_f2 m128 = {128.0f, 128.0f};
    rj_f2 ua, ub, va, vb;
    if constexpr (kHs) {
      const uint32_t u2 = *reinterpret_cast<const uint16_t *>(tu + crow + (x >> 1));
      const uint32_t v2 = *reinterpret_cast<const uint16_t *>(tv + crow + (x >> 1));
      const rj_f2 uu = rj_f2{u8f(u2, 0), u8f(u2, 1)} - m128, vv = rj_f2{u8f(v2, 0), u8f(v2, 1)} - m128;
      ua = rj_f2{uu.x, uu.x};
      ub = rj_f2{uu.y, uu.y};
      va = rj_f2{vv.x, vv.x};
      vb = rj_f2{vv.y, vv.y};
    } else {
      const uint32_t u4 = *reinterpret_cast<const uint32_t *>(tu + crow + x);
      const uint32_t v4 = *reinterpret_cast<const uint32_t *>(tv + crow + x);
      ua = rj_f2{u8f(u4, 0), u8f(u4, 1)} - m128;
      ub = rj_f2{u8f(u4, 2), u8f(u4, 3)} - m128;
      va = rj_f2{u8f(v4, 0), u8f(v4, 1)} - m128;
      vb = rj_f2{u8f(v4, 2), u8f(v4, 3)} - m128;
    }
    uint32_t w0, w1, w2;
    csc4_pk(y4, ua, ub, va, vb, w0, w1, w2);
    const uint32_t off = __umul24(yrow, pitch) + __umul24(qx, 12u);  // 32-bit: saddr store form
    *reinterpret_cast<RJ_GLOBAL uint3 *>(gp(dst) + off) = make_uint3(w0, w1, w2);
    if constexpr (kVs) {  // the second row of the pair, same chroma
      const uint32_t y4b = *reinterpret_cast<const uint32_t *>(ty + __umul24(yrow + 1, tw0) + x);
      csc4_pk(y4b, ua, ub, va, vb, w0, w1, w2);
      *reinterpret_cast<RJ_GLOBAL uint3 *>(gp(dst) + (off + pitch)) = make_uint3(w0, w1, w2);
    }
    qx += qsx;
    qy += qsy;
    if (qx >= quads_x) {
      qx -= quads_x;
      qy++;
    }
  }
}

// Phase C for the commonest strip, 4:2:0 -> RGB over a whole strip of 10 MCUs (160 x 16 px,
// luma tile 160 B wide, chroma tiles 80 B): lane = row pair qy = tid / 8 (8 pairs) and quad
// columns qx = tid % 8 + 8 i, i = 0..4 (40 quads).  Every LDS and global address is the lane's
// base plus a compile-time offset (32 B / 16 B / 96 B per i), so the loop has no address or
// index arithmetic; same pixels, arithmetic and bytes as rgb_strip<true, true>.
__device__ __forceinline__ void rgb_strip_420_full(const uint8_t *ty, const uint8_t *tu, const uint8_t *tv,
                                                   uint32_t tid, uint8_t *dst, uint32_t pitch) {
  const uint32_t qy = tid >> 3, qx0 = tid & 7u;
  const uint8_t *yr = ty + qy * 320u + qx0 * 4u;   // luma rows 2 qy, 2 qy + 1 (tile width 160)
  const uint32_t co = qy * 80u + qx0 * 2u;          // chroma row qy (tile width 80)
  RJ_GLOBAL uint8_t *d = gp(dst) + (__umul24(2u * qy, pitch) + qx0 * 12u);
  const rj_f2 m128 = {128.0f, 128.0f};
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint32_t y4 = *reinterpret_cast<const uint32_t *>(yr + 32 * i);
    const uint32_t y4b = *reinterpret_cast<const uint32_t *>(yr + 160 + 32 * i);
    const uint32_t u2 = *reinterpret_cast<const uint16_t *>(tu + co + 16 * i);
    const uint32_t v2 = *reinterpret_cast<const uint16_t *>(tv + co + 16 * i);
    const rj_f2 uu = rj_f2{u8f(u2, 0), u8f(u2, 1)} - m128, vv = rj_f2{u8f(v2, 0), u8f(v2, 1)} - m128;
    const rj_f2 ua = {uu.x, uu.x}, ub = {uu.y, uu.y}, va = {vv.x, vv.x}, vb = {vv.y, vv.y};
    uint32_t w0, w1, w2;
    csc4_pk(y4, ua, ub, va, vb, w0, w1, w2);
    *reinterpret_cast<RJ_GLOBAL uint3 *>(d + 96 * i) = make_uint3(w0, w1, w2);
    csc4_pk(y4b, ua, ub, va, vb, w0, w1, w2);
    *reinterpret_cast<RJ_GLOBAL uint3 *>(d + pitch + 96 * i) = make_uint3(w0, w1, w2);
  }
}

// The work of one MCU row (one wavefront), looping over the row's strips of S MCUs.
//   kPlanes = false: fused output (rj_decoder.cpp FusedEligible images)
//   kPlanes = true : general path, blocks into the MCU-padded component planes (K2b reads them)
//   kDense = true  : progressive images -- blocks come from the dense coefficient buffer
//                    (rj_prog.hip layout: zigzag, AC sign-magnitude) instead of entry streams
//   kWide = true   : the fix-up pass (k_rows_fix): strips with coefficients outside the int32
//                    IDCT's exact domain take the 64-bit IDCT.  Otherwise such a row is appended
//                    to wide_list (as (image, row); wide_cnt counts) for the fix-up launch.
// The descriptor's byte fields (ncomp .. comp_blk0, bytes [16, 80) of RjImageDev) as 16 dwords.
// Read by wave-uniform dword loads (s_load), so a field is an SALU bit-field extract and a per-lane
// index a select of three words: byte fields read one by one go through the vector memory path,
// each waiting on the one before (the block's component picks its sampling factors), which put
// ~10 dependent memory round trips in front of every row.
struct ImBytes {
  static constexpr uint32_t kBase = 16, kWords = 16;
  uint32_t w[kWords];
  __device__ __forceinline__ explicit ImBytes(const RjImageDev &im) {
    static_assert(offsetof(RjImageDev, ncomp) == kBase && offsetof(RjImageDev, tabset) == kBase + 4 * kWords,
                  "RjImageDev byte fields moved");
    const uint32_t *p = reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(&im) + kBase);
#pragma unroll
    for (uint32_t k = 0; k < kWords; k++) w[k] = p[k];
  }
  // field at a compile-time byte offset
  __device__ __forceinline__ uint32_t at(uint32_t off) const {
    off -= kBase;
    return (w[off >> 2] >> ((off & 3u) * 8u)) & 255u;
  }
  // element `idx` (per lane, < 10) of the byte array at offset `arr`
  __device__ __forceinline__ uint32_t lane_at(uint32_t arr, uint32_t idx) const {
    const uint32_t o = arr - kBase + idx, w0 = (arr - kBase) >> 2, q = (o >> 2) - w0;
    const uint32_t wd = q == 0 ? w[w0] : (q == 1 ? w[w0 + 1] : w[w0 + 2]);
    return (wd >> ((o & 3u) * 8u)) & 255u;
  }
};
#define RJ_OFF(f) uint32_t(offsetof(RjImageDev, f))

template <bool kPlanes, bool kDense, bool kWide = false, bool kSplit = false>
__device__ __forceinline__ void row_body(const RjImageDev *__restrict__ imgs, int i, uint32_t my, RjCoefBuf coefs,
                                         const RjTableSet *__restrict__ tabsets, uint8_t *__restrict__ planes,
                                         uint8_t *s_buf, uint32_t *s_qw, uint32_t *wide_cnt, uint2 *wide_list,
                                         bool only_synced = false) {
  // the main instances dequantise in the entry scatter into the dot2 IDCT's pair layout; the
  // fix-up (kWide) and progressive (kDense) instances keep raw zigzag blocks and the int32 IDCT
  constexpr bool kPairs = !kDense && !kWide;
  uint16_t(*s_q)[64] = reinterpret_cast<uint16_t(*)[64]>(s_qw);
  RJ_STAMP(t_start);
  const uint32_t tid = threadIdx.x;
  const RjImageDev &im = imgs[i];
  const ImBytes ib(im);
  const uint32_t hmax = ib.at(RJ_OFF(hmax)), vmax = ib.at(RJ_OFF(vmax));
  const uint32_t mcu_w = 8 * hmax, mcu_h = 8 * vmax;
  const uint32_t nblk = ib.at(RJ_OFF(nblk_mcu));
  const uint32_t S = U(rj_fused_strip_mcus(hmax, nblk));  // MCUs per strip
  const bool inter = ib.at(RJ_OFF(interleaved)) != 0;
  const uint32_t ncomp = inter ? ib.at(RJ_OFF(ncomp)) : 1;

  // tile geometry (component c: width S*hc*8, height vc*8), all offsets multiples of 8
  uint32_t tw[3], toff[3];
  {
    uint32_t off = 0;
#pragma unroll
    for (int c = 0; c < 3; c++) {
      const bool has = c < int(ncomp);
      const uint32_t hc = (inter && has) ? ib.at(RJ_OFF(comp_h) + c) : 1;
      const uint32_t vc = (inter && has) ? ib.at(RJ_OFF(comp_v) + c) : 1;
      tw[c] = U(S * hc * 8);
      toff[c] = U(off);
      off += has ? tw[c] * vc * 8 : 0;
    }
  }
  // this lane's block inside the strip: component, block column (relative to the strip's first
  // block column of that component) and block row; constant over the row's strips
  uint32_t lane_blk;  // bx | by << 8 | c << 12
  {
    const uint32_t mcu_l = tid / nblk, b_l = tid - mcu_l * nblk;
    const uint32_t c = inter ? ib.lane_at(RJ_OFF(blk_comp), b_l) : 0;
    const uint32_t hc = (ib.w[(RJ_OFF(comp_h) - ImBytes::kBase) >> 2] >> (8u * c)) & 255u;
    const uint32_t bx = mcu_l * (inter ? hc : 1) + (inter ? ib.lane_at(RJ_OFF(blk_dx), b_l) : 0);
    const uint32_t by = inter ? ib.lane_at(RJ_OFF(blk_dy), b_l) : 0;
    lane_blk = (bx & 255u) | (by << 8) | (c << 12);
  }

  const RjTableSet *ts = tabsets + im.tabset;
  if constexpr (kPairs) {
    // s_qw[3 p + c] = quantiser of zigzag position p of component c | its byte offset in the pair
    // layout << 16 (components interleaved: the scatter's ds_read_b32 banks are (a/4) mod 32, and
    // luma and chroma entries of one position then fall in different banks)
    constexpr uint8_t kNatZ[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                   12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                   35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                   58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
    const uint32_t nat = kNatZ[tid];
    const uint32_t slot = rj_pair_slot(nat >> 3, nat & 7) << 16;
    uint32_t q[3];  // loaded unconditionally (the table index is masked): one memory round trip
#pragma unroll
    for (uint32_t c = 0; c < 3; c++) q[c] = ts->qz[ib.at(RJ_OFF(comp_tq) + c) & 3][tid];
#pragma unroll
    for (uint32_t c = 0; c < 3; c++)
      if (c < ncomp) s_qw[3u * tid + c] = q[c] | slot;
  } else {
    uint32_t q[3];
#pragma unroll
    for (uint32_t c = 0; c < 3; c++) q[c] = ts->qz[ib.at(RJ_OFF(comp_tq) + c) & 3][tid];
#pragma unroll
    for (uint32_t c = 0; c < 3; c++)
      if (c < ncomp) s_q[c][tid] = uint16_t(q[c]);
  }

  // this lane's block: LDS base | its component x 4 << 16 (parse_blocks' bpermute source),
  // and its DC quantiser (restore_dc)
  const uint32_t lane_info = tid * RJ_BLK_STRIDE | (lane_blk >> 12) << 18;
  __syncthreads();  // s_qw / s_q written
  const uint32_t q0 = kPairs ? s_qw[lane_blk >> 12] & 0xFFFFu : 0u;
  const uint32_t mcux = U(im.mcux);
  const bool dc_diff = !kDense && U(im.dc_diff) != 0;  // raw entries: restore_dc per strip
  const int thr = int(U(im.idct_thr));
  const uint32_t ri_dc = U(im.ri_mcus ? im.ri_mcus : mcux);
  int carry[3] = {0, 0, 0};
  bool row_wide = false;
  const uint32_t strips_x = (mcux + S - 1) / S;
  const uint32_t *ent = coefs.ent;
  uint32_t cbits = 0;  // component of each block within the MCU
#pragma unroll
  for (uint32_t b = 0; b < RJ_MAX_BLK_MCU; b++)
    if (b < nblk && inter) cbits |= (ib.at(RJ_OFF(blk_comp) + b) & 3u) << (2 * b);
  // the row's first block: its interval, the piece holding it, blocks to skip inside the piece
  Nav nv;
  uint32_t drop = 0;
  EntWin win;
  if constexpr (!kDense) {
    const uint32_t ri = U(im.ri_mcus);
    if (ri == mcux && coefs.seg_lane0 == nullptr) {
      // the row is interval `my`, decoded whole by one exact K1 lane: its single piece sits at
      // the interval's own slot and starts at the row's first block (no segment/piece walk --
      // every load of the row's start is then one dependent step from the row record)
      nv.seg = my;
      nv.pj = 0;
      const RjPiece *p0 = coefs.piece + rj_seg_lane0_k<kSplit>(coefs, U(im.seg_prefix) + my);
      // plain instance in a lean split call (LaunchRows split_rows): a split interval's row is
      // the split-aware launch's
      if (!kSplit && !kWide && coefs.piece_shift != 0 && U(gp(p0)->npieces) == 2u) return;
      // split-aware instance beside it: only the rows whose head met its tail (two pieces); a
      // head that decoded its whole interval left one plain piece, the plain instance's
      if (kSplit && only_synced && U(gp(p0)->npieces) != 2u) return;
      nv.take(p0);
    } else {
      nv.seg = U(ri ? (my * mcux) / ri : 0);
      const RjSegDev sg = gp(im.segs)[nv.seg];
      const uint32_t rel = (my * mcux - sg.mcu_first) * nblk;
      const RjPiece *pb = coefs.piece + rj_seg_lane0_k<kSplit>(coefs, im.seg_prefix + nv.seg);
      const uint32_t np = U(min(gp(pb)->npieces, 4096u));
      uint32_t pj = 0;
      while (pj + 1 < np && U(gp(pb + pj + 1)->first_blk) <= rel) pj++;
      nv.pj = pj;
      nv.take(pb + pj);
      drop = U(rel - gp(pb + pj)->first_blk);
    }
    win.load(ent, nv.cur(), tid);
    win.settle();
  }

  // output descriptor, read once before the strip loop (the output stores could otherwise
  // force re-reads of the descriptor inside the pixel loops)
  uint8_t *const dst0 = im.dst[0], *const dst1 = im.dst[1], *const dst2 = im.dst[2];
  const uint32_t pitch0 = U(im.dst_pitch[0]), pitch1 = U(im.dst_pitch[1]);
  const uint32_t W = U(im.width), H = U(im.height);
  const uint32_t fmt = ib.at(RJ_OFF(fmt));
  const uint32_t hs1 = (ncomp == 3) ? (hmax / ib.at(RJ_OFF(comp_h) + 1) == 2 ? 1u : 0u) : 0u;
  const uint32_t vs1 = (ncomp == 3) ? (vmax / ib.at(RJ_OFF(comp_v) + 1) == 2 ? 1u : 0u) : 0u;
  const bool al_y = ((reinterpret_cast<uintptr_t>(dst0) | pitch0) & 3) == 0;
  const bool al_rgbp = ((reinterpret_cast<uintptr_t>(dst0) | reinterpret_cast<uintptr_t>(dst1) |
                         reinterpret_cast<uintptr_t>(dst2) | pitch0) & 3) == 0;
  const bool al_uv = ((reinterpret_cast<uintptr_t>(dst1) | reinterpret_cast<uintptr_t>(dst2) | pitch1) & 3) == 0;

#ifdef RJ_EXP_STAMPS
  uint64_t acc[4] = {0, 0, 0, 0};
  RJ_STAMP(t_loop);
  acc[3] = t_loop - t_start;
#endif
  for (uint32_t sx = 0; sx < strips_x; sx++) {
    RJ_STAMP(ta);
    const uint32_t mx0 = sx * S;
    const uint32_t nm = min(S, mcux - mx0);
    const uint32_t nb = nm * nblk;
    const bool has_blk = tid < nb;

    bool wide = false;  // some coefficient of the strip needs the exact 64-bit IDCT
    // ---- A: clear the strip's LDS blocks, expand the entry stream into them ----
    __syncthreads();  // previous strip's tiles fully read
    if (!kDense && has_blk) {  // lane b clears block b (compile-time offsets; the dense path overwrites it whole)
      uint4 *z = reinterpret_cast<uint4 *>(s_buf + tid * RJ_BLK_STRIDE);
#pragma unroll
      for (int q = 0; q < 8; q++) z[q] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    if constexpr (kDense) {
      if (has_blk) load_dense_block(im, coefs.dense, lane_blk, mx0, my, inter, s_buf + tid * RJ_BLK_STRIDE);
    } else {
      if (dc_diff)
        parse_blocks<true, kSplit, kPairs>(im, coefs, ent, tid, nb, drop, nblk, cbits, win, nv, s_buf, s_qw, lane_info, thr, wide);
      else
        parse_blocks<false, false, kPairs>(im, coefs, ent, tid, nb, drop, nblk, cbits, win, nv, s_buf, s_qw, lane_info, thr, wide);
      drop = 0;
      if (sx + 1 < strips_x && nv.bleft) win.load(ent, nv.cur(), tid);  // next strip's window: lands behind B and C
    }
    __syncthreads();
    if (!kDense && dc_diff) {
      wide = restore_dc<kPairs>(s_buf, tid, nb, nblk, lane_blk >> 12, mx0, my * mcux, ri_dc, carry, thr, q0) || wide;
      __syncthreads();
    }

    RJ_STAMP(tb);
    RJ_STAMP_ADD(0, tb - ta);
    // ---- B: lane-per-block IDCT in registers ----
    const uint32_t c_b = lane_blk >> 12;
    uint32_t o[16];
    if constexpr (kPairs) {
      uint32_t w[32];
      if (has_blk) {
        const uint4 *src = reinterpret_cast<const uint4 *>(s_buf + tid * RJ_BLK_STRIDE);
#pragma unroll
        for (int q = 0; q < 8; q++) {
          const uint4 a = src[q];
          w[4 * q] = a.x;
          w[4 * q + 1] = a.y;
          w[4 * q + 2] = a.z;
          w[4 * q + 3] = a.w;
        }
      }
      row_wide = row_wide || wide;
      if constexpr (!kPlanes) __syncthreads();  // every block is in registers: the staging area becomes the sample tiles
      if (has_blk) idct_dot2_block(w, o);
      // the next strip's window, before this strip's pixel stores
      if constexpr (!kDense) win.settle();
    } else {
      int32_t v[64];
      const int16_t *zz = reinterpret_cast<const int16_t *>(s_buf + tid * RJ_BLK_STRIDE);
      if (has_blk)
        dezigzag_dequant(reinterpret_cast<const uint4 *>(zz), reinterpret_cast<const uint4 *>(s_q[c_b]), v);
      if constexpr (kDense) {  // progressive coefficients: check the dequantised values directly
        int32_t lo = 0, hi = 0;
#pragma unroll
        for (int k = 0; k < 64; k++) {
          lo = min(lo, v[k]);
          hi = max(hi, v[k]);
        }
        wide = __ballot(has_blk && (lo < -16383 || hi > 16383)) != 0;
      }
      row_wide = row_wide || wide;
      if constexpr (kWide)  // pass 1 now: the tiles overwrite the LDS block below
        if (wide && has_blk) idct_pass1_wide(zz, s_q[c_b], v);
      if constexpr (!kPlanes) __syncthreads();  // every block is in registers: the staging area becomes the sample tiles
      if (has_blk) {
        if (kWide && wide) idct_pass2_wrap(v, o);
        else idct_islow_block(v, o);
      }
    }
    if constexpr (kPlanes) {
      if (has_blk) {
        const uint32_t hc = inter ? im.comp_h[c_b] : 1, vc = inter ? im.comp_v[c_b] : 1;
        const uint32_t bx = mx0 * hc + (lane_blk & 255u), by = my * vc + ((lane_blk >> 8) & 15u);
        const uint32_t pitch = im.plane_pitch[c_b];
        uint8_t *dst = planes + im.plane_off[c_b] + uint64_t(by) * 8u * pitch + bx * 8u;
#pragma unroll
        for (int r = 0; r < 8; r++) *gp(reinterpret_cast<uint2 *>(dst + uint64_t(r) * pitch)) = make_uint2(o[2 * r], o[2 * r + 1]);
      }
      continue;
    }
    if (has_blk) {
      const uint32_t twc = c_b == 0 ? tw[0] : (c_b == 1 ? tw[1] : tw[2]);
      const uint32_t toc = c_b == 0 ? toff[0] : (c_b == 1 ? toff[1] : toff[2]);
      uint8_t *dst = s_buf + toc + ((lane_blk >> 8) & 15u) * 8u * twc + (lane_blk & 255u) * 8u;
#pragma unroll
      for (int r = 0; r < 8; r++) *reinterpret_cast<uint2 *>(dst + r * twc) = make_uint2(o[2 * r], o[2 * r + 1]);
    }
    __syncthreads();

  RJ_STAMP(tc);
  RJ_STAMP_ADD(1, tc - tb);
  // ---- C: output, lane = 4 consecutive pixels ----
  const uint32_t strip_w = nm * mcu_w;
  const uint32_t px0 = mx0 * mcu_w, py0 = my * mcu_h;
  const uint32_t quads_x = strip_w >> 2;  // strip_w is a multiple of 8
  const uint32_t wmax = min(strip_w, W > px0 ? W - px0 : 0u);
  const uint32_t rows = min(mcu_h, H > py0 ? H - py0 : 0u);

  // destination offsets are 32-bit (the host only fuses when pitch * height < 2^31, pitch < 2^24)
  if (fmt == 3 && ncomp == 3 && al_y && wmax == strip_w && rows == mcu_h) {
    const uint8_t *ty = s_buf + toff[0], *tu = s_buf + toff[1], *tv = s_buf + toff[2];
    uint8_t *d = dst0 + (__umul24(py0, pitch0) + px0 * 3);
    if (hs1) {
      if (vs1 && strip_w == 160u && tw[0] == 160u && tw[1] == 80u) {
        rgb_strip_420_full(ty, tu, tv, tid, d, pitch0);
      }
      else if (vs1) rgb_strip<true, true>(ty, tu, tv, tw[0], tw[1], tid, quads_x, rows, d, pitch0);
      else rgb_strip<true, false>(ty, tu, tv, tw[0], tw[1], tid, quads_x, rows, d, pitch0);
    } else {
      if (vs1) rgb_strip<false, true>(ty, tu, tv, tw[0], tw[1], tid, quads_x, rows, d, pitch0);
      else rgb_strip<false, false>(ty, tu, tv, tw[0], tw[1], tid, quads_x, rows, d, pitch0);
    }
  } else if (fmt >= 1 && fmt <= 4) {
    const uint32_t pitch = pitch0;
    const bool a4 = al_y;
    // lane walks quads tid, tid+64, ... of the strip (row-major) with an incremental (x, y)
    const uint32_t qsy = 64 / quads_x, qsx = 64 - qsy * quads_x;
    uint32_t qy = tid / quads_x, qx = tid - qy * quads_x;
    for (; qy < rows; qx += qsx, qy += qsy) {
      if (qx >= quads_x) { qx -= quads_x; qy++; if (qy >= rows) break; }
      const uint32_t y = qy, x = qx * 4;
      if (x >= wmax) continue;
      const uint32_t n = min(4u, wmax - x);
      const uint32_t y4 = *reinterpret_cast<const uint32_t *>(s_buf + toff[0] + __umul24(y, tw[0]) + x);
      const uint32_t py = py0 + y, px = px0 + x;
      if (fmt == 3 || fmt == 4) {
        uint32_t w[3];
        if (ncomp == 3) {
          float u[4], vv[4];
          const uint8_t *ur = s_buf + toff[1] + __umul24(y >> vs1, tw[1]);
          const uint8_t *vr = s_buf + toff[2] + __umul24(y >> vs1, tw[2]);
          if (hs1) {
            const uint32_t u2 = *reinterpret_cast<const uint16_t *>(ur + (x >> 1));
            const uint32_t v2 = *reinterpret_cast<const uint16_t *>(vr + (x >> 1));
            u[0] = u[1] = u8f(u2, 0) - 128.0f;
            u[2] = u[3] = u8f(u2, 1) - 128.0f;
            vv[0] = vv[1] = u8f(v2, 0) - 128.0f;
            vv[2] = vv[3] = u8f(v2, 1) - 128.0f;
          } else {
            const uint32_t u4 = *reinterpret_cast<const uint32_t *>(ur + x);
            const uint32_t v4 = *reinterpret_cast<const uint32_t *>(vr + x);
#pragma unroll
            for (int j = 0; j < 4; j++) {
              u[j] = u8f(u4, j) - 128.0f;
              vv[j] = u8f(v4, j) - 128.0f;
            }
          }
          csc4(y4, u, vv, w[0], w[1], w[2]);
        } else {  // 4:0:0 -> R = G = B = Y (rocjpeg_hip_kernels.cpp:1874-1932)
          const uint32_t b0 = y4 & 255, b1 = (y4 >> 8) & 255, b2 = (y4 >> 16) & 255, b3 = y4 >> 24;
          w[0] = b0 | (b0 << 8) | (b0 << 16) | (b1 << 24);
          w[1] = b1 | (b1 << 8) | (b2 << 16) | (b2 << 24);
          w[2] = b2 | (b3 << 8) | (b3 << 16) | (b3 << 24);
        }
        if (fmt == 3) {
          uint8_t *d = dst0 + (__umul24(py, pitch) + px * 3);
          if (n == 4 && a4) {
            *gp(reinterpret_cast<uint3 *>(d)) = make_uint3(w[0], w[1], w[2]);
          } else {
            store_bytes(d, 3 * n, w);
          }
        } else {  // RGB planar: R, G, B planes, all with pitch[0] (rocjpeg_decoder.cpp:525-544)
          // byte k of w = pixel k/3, channel k%3
          const uint32_t R = (w[0] & 0xFFu) | ((w[0] >> 16) & 0xFF00u) | (w[1] & 0xFF0000u) | ((w[2] << 16) & 0xFF000000u);
          const uint32_t G = ((w[0] >> 8) & 0xFFu) | ((w[1] << 8) & 0xFF00u) | ((w[1] >> 8) & 0xFF0000u) |
                             ((w[2] << 8) & 0xFF000000u);
          const uint32_t B = ((w[0] >> 16) & 0xFFu) | (w[1] & 0xFF00u) | ((w[2] << 16) & 0xFF0000u) | (w[2] & 0xFF000000u);
          const uint32_t pl[3] = {R, G, B};
          const bool ap = al_rgbp;
          const uint32_t off = __umul24(py, pitch) + px;
#pragma unroll
          for (int p = 0; p < 3; p++) {
            uint8_t *d = (p == 0 ? dst0 : (p == 1 ? dst1 : dst2)) + off;
            if (n == 4 && ap) *gp(reinterpret_cast<uint32_t *>(d)) = pl[p];
            else store_bytes(d, n, &pl[p]);
          }
        }
      } else {  // Y plane (OUTPUT_Y, and the luma of YUV_PLANAR)
        uint8_t *d = dst0 + (__umul24(py, pitch) + px);
        if (n == 4 && a4) *gp(reinterpret_cast<uint32_t *>(d)) = y4;
        else store_bytes(d, n, &y4);
      }
    }
  }
  if (fmt == 1 && ncomp == 3) {  // YUV_PLANAR chroma planes at native resolution; U and V share pitch[1]
    const bool a4 = al_uv;
    const uint32_t cW = hs1 ? (W >> 1) : W, cH = vs1 ? (H >> 1) : H;
    const uint32_t cw = strip_w >> hs1, ch = mcu_h >> vs1;
    const uint32_t cx0 = px0 >> hs1, cy0 = py0 >> vs1;
    const uint32_t cq = cw >> 2;
    const uint32_t cwmax = min(cw, cW > cx0 ? cW - cx0 : 0u);
    const uint32_t crows = min(ch, cH > cy0 ? cH - cy0 : 0u);
    // lane walks quads tid, tid + 64, ... of the U plane's strip, then of the V plane's, with an
    // incremental (row, quad) (a division only at the start and where it enters the V plane)
    const uint32_t cqd = max(cq, 1u);  // (no iteration when cq = 0)
    const uint32_t tot = cq * crows, csy = 64 / cqd, csx = 64 - csy * cqd;
    uint32_t second = 0, y = tid / cqd, xq = tid - y * cqd;
    for (uint32_t k = tid; k < 2 * tot; k += 64, xq += csx, y += csy) {
      if (xq >= cq) {
        xq -= cq;
        y++;
      }
      if (second == 0 && k >= tot) {
        second = 1;
        y = (k - tot) / cqd;
        xq = (k - tot) - y * cqd;
      }
      const uint32_t x = xq * 4;
      if (x >= cwmax) continue;
      const uint32_t n = min(4u, cwmax - x);
      const uint32_t s4 = *reinterpret_cast<const uint32_t *>(s_buf + (second ? toff[2] : toff[1]) +
                                                              __umul24(y, second ? tw[2] : tw[1]) + x);
      uint8_t *d = (second ? dst2 : dst1) + (__umul24(cy0 + y, pitch1) + cx0 + x);
      if (n == 4 && a4) *gp(reinterpret_cast<uint32_t *>(d)) = s4;
      else store_bytes(d, n, &s4);
    }
  }
  RJ_STAMP(te);
  RJ_STAMP_ADD(2, te - tc);
  }  // strips
  if constexpr (!kWide)
    if (row_wide && tid == 0) {
      // (the launches sharing one list decode disjoint rows; the bound keeps a miscount from
      // spilling into the next list)
      const uint32_t k = atomicAdd(wide_cnt, 1u);
      if (k < coefs.wide_cap) wide_list[k] = make_uint2(uint32_t(i), my);
      // host-mapped flag: the host issues the fix-up launches after the call's kernels
      __hip_atomic_store(coefs.wide_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#ifdef RJ_EXP_STAMPS
  if (tid == 0)
    for (int q = 0; q < 4; q++) atomicAdd(&rj_stamp[q], (unsigned long long)acc[q]);
  if (tid == 0) atomicAdd(&rj_stamp[4], 1ull);
#endif
}

// K2: one wavefront (workgroup) per MCU row.
template <bool kPlanes, bool kDense = false, bool kSplit = false>
__global__ __launch_bounds__(64, RJ_K2_OCC) void k_rows(const RjImageDev *__restrict__ imgs, int nimg,
                                             const uint32_t *__restrict__ row_prefix,
                                             const uint2 *__restrict__ row_list,
                                             RjCoefBuf coefs,
                                             const RjTableSet *__restrict__ tabsets,
                                             uint8_t *__restrict__ planes, uint32_t *wide_cnt, uint2 *wide_list) {
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[RJ_FUSED_MAX_BLK * RJ_BLK_STRIDE];  // A/B, then tiles
  __shared__ __attribute__((aligned(16))) uint32_t s_qw[3 * 64];
  int i;
  uint32_t my;
  row_of_block(imgs, nimg, row_prefix, row_list, blockIdx.x, i, my);
  row_body<kPlanes, kDense, false, kSplit>(imgs, i, my, coefs, tabsets, planes, s_buf, s_qw, wide_cnt, wide_list);
}

// K2 of lean split calls' rows (pieces, skips, early-ending tails) with its own register budget
template <bool kPlanes>
__global__ __launch_bounds__(64, RJ_K2_SPLIT_OCC) void k_rows_split(const RjImageDev *__restrict__ imgs, int nimg,
                                                                   const uint32_t *__restrict__ row_prefix,
                                                                   const uint2 *__restrict__ row_list, RjCoefBuf coefs,
                                                                   const RjTableSet *__restrict__ tabsets,
                                                                   uint8_t *__restrict__ planes, uint32_t *wide_cnt,
                                                                   uint2 *wide_list, uint32_t only_synced) {
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[RJ_FUSED_MAX_BLK * RJ_BLK_STRIDE];
  __shared__ __attribute__((aligned(16))) uint32_t s_qw[3 * 64];
  int i;
  uint32_t my;
  row_of_block(imgs, nimg, row_prefix, row_list, blockIdx.x, i, my);
  row_body<kPlanes, false, false, true>(imgs, i, my, coefs, tabsets, planes, s_buf, s_qw, wide_cnt, wide_list,
                                        only_synced != 0);
}

// K2 of progressive images (dense coefficients, int32 IDCT) with its own register budget
template <bool kPlanes>
__global__ __launch_bounds__(64, RJ_K2_DENSE_OCC) void k_rows_dense(const RjImageDev *__restrict__ imgs, int nimg,
                                                                   const uint32_t *__restrict__ row_prefix,
                                                                   const uint2 *__restrict__ row_list, RjCoefBuf coefs,
                                                                   const RjTableSet *__restrict__ tabsets,
                                                                   uint8_t *__restrict__ planes, uint32_t *wide_cnt,
                                                                   uint2 *wide_list) {
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[RJ_FUSED_MAX_BLK * RJ_BLK_STRIDE];
  __shared__ __attribute__((aligned(16))) uint32_t s_qw[3 * 64];
  int i;
  uint32_t my;
  row_of_block(imgs, nimg, row_prefix, row_list, blockIdx.x, i, my);
  row_body<kPlanes, true, false, false>(imgs, i, my, coefs, tabsets, planes, s_buf, s_qw, wide_cnt, wide_list);
}

// ---- live rows (rj_device.h RjLive): K2 beside K1 ----
#define RJ_LIVE_RESIDENT_TICKS 2000ull   // 20 us (s_memrealtime, 100 MHz): K1 must be resident by then
#define RJ_LIVE_ROW_TICKS 400000000ull   // 4 s: a published row never takes this long (defence only)
#ifndef RJ_LIVE_POLL
#define RJ_LIVE_POLL 16                   // s_sleep between polls of a waiting live workgroup (x 64 cycles)
#endif
__device__ __forceinline__ uint32_t live_ld(uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// lane 0: a ticket's published slot (epoch | row << 32), or 0 (leave: K1 not resident in time,
// the ticket counter closed by K1's last wave, or the ticket past every published row)
__device__ __forceinline__ unsigned long long live_claim(const RjLive &lv, uint32_t *host_flag) {
  uint32_t *c = lv.ctr;
  if (live_ld(c + RJ_LIVE_GIVEUP) != 0u || live_ld(c + RJ_LIVE_DONE) >= lv.k1_waves) return 0;
  // waiting on a row is safe only once every K1 workgroup holds its CU: a K2 workgroup that
  // arrived first would otherwise keep a K1 workgroup from its LDS
  const uint64_t t0 = wall_clock64();
  while (live_ld(c + RJ_LIVE_STARTED) < lv.k1_groups) {
    if (wall_clock64() - t0 > RJ_LIVE_RESIDENT_TICKS) {
      __hip_atomic_store(c + RJ_LIVE_GIVEUP, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return 0;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  // only on a CU whose K1 workgroup is done: beside a running one, this wave's LDS and issue
  // traffic lengthens K1's symbol chains (measured: K1 1.7 -> 2.9 ms)
  {
    const uint32_t *busy = lv.cu_busy + rj_live_cu_key();
    while (__hip_atomic_load(busy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
      if (live_ld(c + RJ_LIVE_DONE) >= lv.k1_waves) return 0;  // K1 is over: k_rows_rest takes the rest
      __builtin_amdgcn_s_sleep(RJ_LIVE_POLL);
    }
  }
  const uint32_t t = atomicAdd(c + RJ_LIVE_TICKET, 1u);
  if ((t & RJ_LIVE_CLOSED) != 0u || t >= lv.rows) return 0;
  unsigned long long *sp = lv.slot + t;
  const uint64_t t1 = wall_clock64();
  for (;;) {
    unsigned long long v = __hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (uint32_t(v) == lv.epoch) return v;
    if (live_ld(c + RJ_LIVE_DONE) >= lv.k1_waves) {  // every slot K1 reserved is written by now
      v = __hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return uint32_t(v) == lv.epoch ? v : 0ull;
    }
    if (wall_clock64() - t1 > RJ_LIVE_ROW_TICKS) {  // the row is lost: the host re-decodes the call's rows
      __hip_atomic_store(c + RJ_LIVE_ERROR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(host_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return 0;
    }
    __builtin_amdgcn_s_sleep(RJ_LIVE_POLL);
  }
}

// K2 beside K1 (a second, low-priority stream): one workgroup per row K1 may publish; it decodes
// the row its ticket names once K1 has published it (agent-scope acquire: the guide's valid
// consumer form -- one relaxed poll, one acquire, then plain loads).
__global__ __launch_bounds__(64, RJ_K2_OCC) void k_rows_live(const RjImageDev *__restrict__ imgs, int nimg, RjLive lv,
                                                          RjCoefBuf coefs, const RjTableSet *__restrict__ tabsets,
                                                          uint32_t *wide_cnt, uint2 *wide_list) {
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[RJ_FUSED_MAX_BLK * RJ_BLK_STRIDE];
  __shared__ __attribute__((aligned(16))) uint32_t s_qw[3 * 64];
  unsigned long long v = 0;
  if (threadIdx.x == 0) v = live_claim(lv, coefs.wide_flag + 1);
  const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(v >> 32));
  const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(v));
  if (lo == 0u) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int i = int(hi >> RJ_LIVE_ROW_BITS);
  if (i >= nimg) return;
  row_body<false, false, false, false>(imgs, i, hi & ((1u << RJ_LIVE_ROW_BITS) - 1u), coefs, tabsets, nullptr, s_buf,
                                       s_qw, wide_cnt, wide_list);
}

// K2 after K1 (stream order): the published rows no ticket took -- [min(final tickets,
// published), published); K1's last wave closed the ticket counter and stored its final value.
__global__ __launch_bounds__(64, RJ_K2_OCC) void k_rows_rest(const RjImageDev *__restrict__ imgs, int nimg, RjLive lv,
                                                          RjCoefBuf coefs, const RjTableSet *__restrict__ tabsets,
                                                          uint32_t *wide_cnt, uint2 *wide_list) {
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[RJ_FUSED_MAX_BLK * RJ_BLK_STRIDE];
  __shared__ __attribute__((aligned(16))) uint32_t s_qw[3 * 64];
  const uint32_t pub = min(U(lv.ctr[RJ_LIVE_RESERVED]), lv.rows);
  const uint32_t pos = min(U(lv.ctr[RJ_LIVE_FINAL]), pub) + blockIdx.x;
  if (pos >= pub) return;
  const unsigned long long v = lv.slot[pos];
  const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(v >> 32));
  if (__builtin_amdgcn_readfirstlane(uint32_t(v)) != lv.epoch) {  // never expected: K1 published it
    if (threadIdx.x == 0) __hip_atomic_store(coefs.wide_flag + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  const int i = int(hi >> RJ_LIVE_ROW_BITS);
  if (i >= nimg) return;
  row_body<false, false, false, false>(imgs, i, hi & ((1u << RJ_LIVE_ROW_BITS) - 1u), coefs, tabsets, nullptr, s_buf,
                                       s_qw, wide_cnt, wide_list);
}

hipError_t LaunchRowsLive(hipStream_t st, const RjImageDev *imgs, int nimg, const RjLive &lv, RjCoefBuf coefs,
                          const RjTableSet *tabsets, uint32_t *wide_cnt, uint2 *wide_list, uint32_t extra_lds) {
  if (lv.rows == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rows_live, dim3(lv.rows), dim3(64), extra_lds, st, imgs, nimg, lv, coefs, tabsets, wide_cnt,
                     wide_list);
  return hipGetLastError();
}

hipError_t LaunchRowsRest(hipStream_t st, const RjImageDev *imgs, int nimg, const RjLive &lv, RjCoefBuf coefs,
                          const RjTableSet *tabsets, uint32_t *wide_cnt, uint2 *wide_list) {
  if (lv.rows == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rows_rest, dim3(lv.rows), dim3(64), 0, st, imgs, nimg, lv, coefs, tabsets, wide_cnt, wide_list);
  return hipGetLastError();
}

hipError_t LaunchRowsSplit(hipStream_t st, const RjImageDev *imgs, int nimg, const uint2 *split_rows,
                           uint32_t nsplit_rows, RjCoefBuf coefs, const RjTableSet *tabsets, uint32_t *wide_cnt,
                           uint2 *wide_list) {
  if (nsplit_rows == 0 || split_rows == nullptr) return hipSuccess;
  const uint32_t *no_prefix = nullptr;
  uint8_t *no_planes = nullptr;
  hipLaunchKernelGGL(k_rows_split<false>, dim3(nsplit_rows), dim3(64), 0, st, imgs, nimg, no_prefix, split_rows, coefs,
                     tabsets, no_planes, wide_cnt, wide_list, 1u);
  return hipGetLastError();
}

// K2 fix-up: the rows a K2 launch recorded (a strip outside the int32 IDCT's exact domain --
// corrupt data with large quantisers), decoded again with the 64-bit IDCT for those strips.
// Issued by the host only when a K2 launch of the call raised the host-mapped flag
// (RjCoefBuf.wide_flag), after the call's kernels -- the common path pays nothing.
template <bool kPlanes, bool kDense, bool kSplit = false>
__global__ __launch_bounds__(64) void k_rows_fix(const RjImageDev *__restrict__ imgs, int nimg, RjCoefBuf coefs,
                                                 const RjTableSet *__restrict__ tabsets, uint8_t *__restrict__ planes,
                                                 const uint32_t *wide_cnt, const uint2 *wide_list, uint32_t cap) {
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[RJ_FUSED_MAX_BLK * RJ_BLK_STRIDE];
  __shared__ __attribute__((aligned(16))) uint32_t s_qw[3 * 64];
  const uint32_t cnt = min(U(*wide_cnt), cap);
  for (uint32_t r = blockIdx.x; r < cnt; r += gridDim.x) {
    const uint2 e = wide_list[r];
    const int i = int(U(e.x));
    if (i >= nimg) continue;
    __syncthreads();  // the previous row's tiles fully read
    row_body<kPlanes, kDense, true, kSplit>(imgs, i, U(e.y), coefs, tabsets, planes, s_buf, s_qw, nullptr, nullptr);
  }
}

// the fix-up launch behind a K2 launch of `cap` rows (same stream, same variant; a lean split
// launch's pieces, coefs.piece_shift = 1, take the split-aware instances)
hipError_t LaunchRowsFix(hipStream_t st, bool to_planes, bool dense, const RjImageDev *imgs, int nimg, RjCoefBuf coefs,
                         const RjTableSet *tabsets, uint8_t *planes, const uint32_t *wide_cnt, const uint2 *wide_list,
                         uint32_t cap) {
  if (cap == 0) return hipSuccess;
  const dim3 grid(std::min<uint32_t>(cap, 256));
  if (dense) {
    if (to_planes)
      hipLaunchKernelGGL((k_rows_fix<true, true>), grid, dim3(64), 0, st, imgs, nimg, coefs, tabsets, planes, wide_cnt, wide_list, cap);
    else
      hipLaunchKernelGGL((k_rows_fix<false, true>), grid, dim3(64), 0, st, imgs, nimg, coefs, tabsets, planes, wide_cnt, wide_list, cap);
  } else if (coefs.piece_shift != 0) {
    if (to_planes)
      hipLaunchKernelGGL((k_rows_fix<true, false, true>), grid, dim3(64), 0, st, imgs, nimg, coefs, tabsets, planes, wide_cnt, wide_list, cap);
    else
      hipLaunchKernelGGL((k_rows_fix<false, false, true>), grid, dim3(64), 0, st, imgs, nimg, coefs, tabsets, planes, wide_cnt, wide_list, cap);
  } else {
    if (to_planes)
      hipLaunchKernelGGL((k_rows_fix<true, false>), grid, dim3(64), 0, st, imgs, nimg, coefs, tabsets, planes, wide_cnt, wide_list, cap);
    else
      hipLaunchKernelGGL((k_rows_fix<false, false>), grid, dim3(64), 0, st, imgs, nimg, coefs, tabsets, planes, wide_cnt, wide_list, cap);
  }
  return hipGetLastError();
}

hipError_t LaunchRows(hipStream_t st, bool to_planes, const RjImageDev *imgs, int nimg, const uint32_t *row_prefix,
                      const uint2 *row_list, uint32_t nrows, RjCoefBuf coefs, const RjTableSet *tabsets,
                      uint8_t *planes, uint32_t *wide_cnt, uint2 *wide_list, const uint2 *split_rows,
                      uint32_t nsplit_rows, hipStream_t split_st) {
  if (nrows == 0) return hipSuccess;
  if (coefs.piece_shift != 0 && split_rows != nullptr) {  // plain rows, then the split intervals' rows
    const uint32_t *no_prefix = nullptr;
    hipStream_t sst = split_st != nullptr ? split_st : st;
    if (to_planes) {
      hipLaunchKernelGGL(k_rows<true>, dim3(nrows), dim3(64), 0, st, imgs, nimg, row_prefix, row_list, coefs, tabsets,
                         planes, wide_cnt, wide_list);
      if (nsplit_rows)
        hipLaunchKernelGGL(k_rows_split<true>, dim3(nsplit_rows), dim3(64), 0, sst, imgs, nimg, no_prefix,
                           split_rows, coefs, tabsets, planes, wide_cnt, wide_list, 1u);
    } else {
      hipLaunchKernelGGL(k_rows<false>, dim3(nrows), dim3(64), 0, st, imgs, nimg, row_prefix, row_list, coefs, tabsets,
                         planes, wide_cnt, wide_list);
      if (nsplit_rows)
        hipLaunchKernelGGL(k_rows_split<false>, dim3(nsplit_rows), dim3(64), 0, sst, imgs, nimg, no_prefix,
                           split_rows, coefs, tabsets, planes, wide_cnt, wide_list, 1u);
    }
  } else if (coefs.piece_shift != 0) {  // lean split launch: pieces with skips / early terminators
    if (to_planes)
      hipLaunchKernelGGL(k_rows_split<true>, dim3(nrows), dim3(64), 0, st, imgs, nimg, row_prefix, row_list,
                         coefs, tabsets, planes, wide_cnt, wide_list, 0u);
    else
      hipLaunchKernelGGL(k_rows_split<false>, dim3(nrows), dim3(64), 0, st, imgs, nimg, row_prefix, row_list,
                         coefs, tabsets, planes, wide_cnt, wide_list, 0u);
  } else if (to_planes) {
    hipLaunchKernelGGL(k_rows<true>, dim3(nrows), dim3(64), 0, st, imgs, nimg, row_prefix, row_list, coefs,
                       tabsets, planes, wide_cnt, wide_list);
  } else {
    hipLaunchKernelGGL(k_rows<false>, dim3(nrows), dim3(64), 0, st, imgs, nimg, row_prefix, row_list, coefs,
                       tabsets, planes, wide_cnt, wide_list);
  }
  return hipGetLastError();
}

hipError_t LaunchRowsDense(hipStream_t st, bool to_planes, const RjImageDev *imgs, int nimg, const uint32_t *row_prefix,
                           uint32_t nrows, RjCoefBuf coefs, const RjTableSet *tabsets, uint8_t *planes,
                           uint32_t *wide_cnt, uint2 *wide_list) {
  if (nrows == 0) return hipSuccess;
  const uint2 *no_list = nullptr;
  if (to_planes)
    hipLaunchKernelGGL(k_rows_dense<true>, dim3(nrows), dim3(64), 0, st, imgs, nimg, row_prefix, no_list, coefs,
                       tabsets, planes, wide_cnt, wide_list);
  else
    hipLaunchKernelGGL(k_rows_dense<false>, dim3(nrows), dim3(64), 0, st, imgs, nimg, row_prefix, no_list, coefs,
                       tabsets, planes, wide_cnt, wide_list);
  return hipGetLastError();
}

#ifdef RJ_EXP_STAMPS
void DumpRowStamps() {
  unsigned long long h[8];
  (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(rj_stamp), sizeof(h));
  const double w = h[4] ? double(h[4]) : 1.0;
  fprintf(stderr, "[rj stamps] waves %llu  per wave cycles: A %.0f B %.0f C %.0f prologue %.0f\n", h[4], h[0] / w,
          h[1] / w, h[2] / w, h[3] / w);
  unsigned long long z[8] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(rj_stamp), z, sizeof(z));
}
#endif

}  // namespace rj
