// rj_math.h -- per-element arithmetic of the decode path, shared by the general and the
// fused kernels so both produce identical bytes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rj_device.h"

namespace rj {

// Global-address-space views of generic pointers.  Pointers read from descriptors are generic,
// and the backend then emits FLAT memory instructions, which count in lgkmcnt as well as
// vmcnt: every later s_waitcnt on an LDS read would also wait for those stores to reach
// memory.  Every global access in the kernels goes through these (global_* instructions).
#if defined(__HIP_DEVICE_COMPILE__)
#define RJ_GLOBAL __attribute__((address_space(1)))
#else
#define RJ_GLOBAL  // host pass of the single-source build: never executed
#endif
template <typename T>
__device__ __forceinline__ RJ_GLOBAL T *gp(T *p) {
  return (RJ_GLOBAL T *)p;
}
template <typename T>
__device__ __forceinline__ const RJ_GLOBAL T *gp(const T *p) {
  return (const RJ_GLOBAL T *)p;
}

// libjpeg ISLOW constants (jidctint.c: CONST_BITS 13, PASS1_BITS 2).  Computed in int32
// with 24-bit multiplies (v_mul_i32_i24, full rate; v_mul_lo_u32 is quarter rate): exact --
// i.e. equal to libjpeg's wide arithmetic -- whenever every dequantised coefficient has
// |x| < 2^14, which every stream produced from an 8-bit DCT satisfies (|x| <= ~2^11 * 8);
// then every multiplicand is < 2^17 and every product and sum fits int32.  libjpeg-turbo's
// SIMD ISLOW kernels make the same (in fact a 16-bit) assumption.
#define RJ_FIX_0_298631336 2446
#define RJ_FIX_0_390180644 3196
#define RJ_FIX_0_541196100 4433
#define RJ_FIX_0_765366865 6270
#define RJ_FIX_0_899976223 7373
#define RJ_FIX_1_175875602 9633
#define RJ_FIX_1_501321110 12299
#define RJ_FIX_1_847759065 15137
#define RJ_FIX_1_961570560 16069
#define RJ_FIX_2_053119869 16819
#define RJ_FIX_2_562915447 20995
#define RJ_FIX_3_072711026 25172

__device__ __forceinline__ int32_t m24(int32_t a, int32_t k) { return __mul24(a, k); }

// K1 lane layout lookups (RjCoefBuf); null tables mean the identity layout
__device__ __forceinline__ uint32_t rj_lane_seg(const RjCoefBuf &c, uint32_t lane) {
  return c.lane_seg ? *gp(c.lane_seg + lane) : lane;
}
__device__ __forceinline__ uint32_t rj_seg_lane0(const RjCoefBuf &c, uint32_t seg) {
  return c.seg_lane0 ? *gp(c.seg_lane0 + seg) : seg << c.piece_shift;
}
// the same where the kernel instance knows the layout (kSplit: a lean split launch, piece_shift 1)
template <bool kSplit>
__device__ __forceinline__ uint32_t rj_seg_lane0_k(const RjCoefBuf &c, uint32_t seg) {
  return c.seg_lane0 ? *gp(c.seg_lane0 + seg) : (kSplit ? seg << 1 : seg << c.piece_shift);
}

// Inclusive prefix sum over the wave's 64 lanes (DPP: row shifts, then row broadcasts; gfx9).
__device__ __forceinline__ int wave_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return x;
}
// lane l gets lane l - 1's x (lane 0: 0) / lane l + 1's x (lane 63: 0): DPP wave_shr:1 / wave_shl:1
__device__ __forceinline__ uint32_t wave_prev(uint32_t x) {
  return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ uint32_t wave_next(uint32_t x) {
  return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x130, 0xF, 0xF, false));
}

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

// One 8-point ISLOW butterfly on x0..x7 (dequantised coefficients or pass-1 outputs).  `rnd`
// is added to the even part, so it reaches all eight outputs: callers fold the descale
// rounding (and the range-limit offset) into it.  Writes the pre-shift sums t[0..7].
__device__ __forceinline__ void islow_1d(int32_t x0, int32_t x1, int32_t x2, int32_t x3, int32_t x4, int32_t x5,
                                         int32_t x6, int32_t x7, int32_t rnd, int32_t t[8]) {
  int32_t z1 = m24(x2 + x6, RJ_FIX_0_541196100);
  const int32_t tmp2 = z1 - m24(x6, RJ_FIX_1_847759065);
  const int32_t tmp3 = z1 + m24(x2, RJ_FIX_0_765366865);
  const int32_t e0 = ((x0 + x4) << 13) + rnd, e1 = ((x0 - x4) << 13) + rnd;
  const int32_t t10 = e0 + tmp3, t13 = e0 - tmp3, t11 = e1 + tmp2, t12 = e1 - tmp2;
  int32_t o0 = x7, o1 = x5, o2 = x3, o3 = x1;
  z1 = o0 + o3;
  int32_t z2 = o1 + o2, z3 = o0 + o2, z4 = o1 + o3;
  const int32_t z5 = m24(z3 + z4, RJ_FIX_1_175875602);
  o0 = m24(o0, RJ_FIX_0_298631336);
  o1 = m24(o1, RJ_FIX_2_053119869);
  o2 = m24(o2, RJ_FIX_3_072711026);
  o3 = m24(o3, RJ_FIX_1_501321110);
  z1 = m24(z1, -RJ_FIX_0_899976223);
  z2 = m24(z2, -RJ_FIX_2_562915447);
  z3 = m24(z3, -RJ_FIX_1_961570560) + z5;
  z4 = m24(z4, -RJ_FIX_0_390180644) + z5;
  o0 += z1 + z3;
  o1 += z2 + z4;
  o2 += z2 + z3;
  o3 += z1 + z4;
  t[0] = t10 + o3;
  t[7] = t10 - o3;
  t[1] = t11 + o2;
  t[6] = t11 - o2;
  t[2] = t12 + o1;
  t[5] = t12 - o1;
  t[3] = t13 + o0;
  t[4] = t13 - o0;
}

// Expand one block's sparse entries (16-B aligned list, `cnt` valid) into a zeroed 128-B LDS
// block in zigzag order.  Two 16-B loads in flight per step.
__device__ __forceinline__ void scatter_block(const uint4 *src, uint32_t cnt, int16_t *dst_zz) {
  const uint32_t nq = (cnt + 3) >> 2;
  for (uint32_t q = 0; q < nq; q += 2) {
    const uint4 a = src[q];
    const uint4 b = (q + 1 < nq) ? src[q + 1] : make_uint4(0, 0, 0, 0);
    const uint32_t e[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int j = 0; j < 8; j++)
      if (4 * q + j < cnt) dst_zz[(e[j] >> 16) & 63] = int16_t(e[j] & 0xFFFF);
  }
}

// K1 stores each block in zigzag order (its decode order); the quant tables are also kept in
// zigzag (DQT) order, so dequantisation is element-wise and the permutation to natural order
// happens in registers with compile-time indices.
__device__ __forceinline__ void dezigzag_dequant(const uint4 *coef_zz, const uint4 *q_zz, int32_t (&v)[64]) {
  constexpr uint8_t kNat[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const uint4 a = coef_zz[r], qa = q_zz[r];
    const uint32_t aw[4] = {a.x, a.y, a.z, a.w}, qw[4] = {qa.x, qa.y, qa.z, qa.w};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      v[kNat[r * 8 + 2 * j]] = int32_t(int16_t(aw[j] & 0xFFFF)) * int32_t(qw[j] & 0xFFFF);
      v[kNat[r * 8 + 2 * j + 1]] = int32_t(int16_t(aw[j] >> 16)) * int32_t(qw[j] >> 16);
    }
  }
}

// libjpeg range_limit[DESCALE(t, 18) & RANGE_MASK] (+CENTERJSAMPLE folded in) for a pass-2
// sum t that already carries RJ_PASS2_RND: bits 18..27 are ((DESCALE(t) + 512) & 1023) = w,
// the sample is clamp(w - 384, 0, 255).  Returned as med3(w, 384, 639), whose low byte XOR
// 0x80 is that sample (384 = 0x180): four of them pack with v_perm + one XOR.
#define RJ_PASS1_RND (1 << 10)
#define RJ_PASS2_RND ((1 << 17) + (512 << 18))
__device__ __forceinline__ uint32_t islow_limit_biased(int32_t t) {
  const uint32_t w = __builtin_amdgcn_ubfe(uint32_t(t), 18, 10);
  return min(max(w, 384u), 639u);  // v_med3_u32
}
__device__ __forceinline__ uint32_t islow_pack4(uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3) {
  const uint32_t p01 = __builtin_amdgcn_perm(m1, m0, 0x0c0c0400u);
  const uint32_t p23 = __builtin_amdgcn_perm(m3, m2, 0x0c0c0400u);
  return __builtin_amdgcn_perm(p23, p01, 0x05040100u) ^ 0x80808080u;
}
// pass 1 (columns) on v in place, then pass 2 (rows): row r of samples -> o[2r] (x 0..3),
// o[2r+1] (x 4..7), little-endian bytes.
__device__ __forceinline__ void idct_islow_block(int32_t (&v)[64], uint32_t (&o)[16]) {
#pragma unroll
  for (int c = 0; c < 8; c++) {
    int32_t t[8];
    islow_1d(v[c], v[8 + c], v[16 + c], v[24 + c], v[32 + c], v[40 + c], v[48 + c], v[56 + c], RJ_PASS1_RND, t);
#pragma unroll
    for (int r = 0; r < 8; r++) v[r * 8 + c] = t[r] >> 11;  // DESCALE(, CONST_BITS-PASS1_BITS)
  }
#pragma unroll
  for (int r = 0; r < 8; r++) {
    int32_t t[8];
    islow_1d(v[r * 8], v[r * 8 + 1], v[r * 8 + 2], v[r * 8 + 3], v[r * 8 + 4], v[r * 8 + 5], v[r * 8 + 6],
             v[r * 8 + 7], RJ_PASS2_RND, t);
    o[2 * r] = islow_pack4(islow_limit_biased(t[0]), islow_limit_biased(t[1]), islow_limit_biased(t[2]),
                           islow_limit_biased(t[3]));
    o[2 * r + 1] = islow_pack4(islow_limit_biased(t[4]), islow_limit_biased(t[5]), islow_limit_biased(t[6]),
                               islow_limit_biased(t[7]));
  }
}

// ---- ISLOW with packed 16-bit dot products (v_dot2c_i32_i16) ----
// Every output of one ISLOW pass is an integer linear combination of its 8 inputs (the
// butterfly above only multiplies by constants and adds), t[r] = sum_k A[r][k] x[k] with
//   A[r][k] = 8192 (k = 0), and +-{11363, 10703, 9633, 8192, 6437, 4433, 2260} -- all int16,
// and t[r] / t[7-r] share the even part (x0, x2, x4, x6) and negate the odd part.  So a pass is
// 14 dot2 + 8 add/sub on packed input pairs instead of 12 multiplies + ~26 adds on int32, with
// the inputs in registers at half the width.  Pair layout of a block (32 dwords, built by
// K2's entry scatter straight into LDS, see rj_pair_slot): dword 4c + j of column c holds
//   j = 0: (x0, x4), 1: (x2, x6), 2: (x1, x3), 3: (x5, x7)   (low half, high half)
// Scaling: the scatter stores the dequantised coefficient x 32 (the DC x 16, its constant
// 16384), so a pass-1 sum is 32 x (t + 1024) and DESCALE(t, 11) is its high half: the pass-2
// pairs are packed by one v_perm per two outputs, no shifts.  Pass 2 needs only bits 18..27 of
// its sums (range-limit mask), which wrap-around int32 arithmetic keeps exact.
// Exact -- equal to libjpeg's wide arithmetic -- whenever every pass-1 output fits int16; the
// fast domain K2 checks per coefficient is |DC| <= 1151 and |AC| <= 1023 (dequantised), for
// which |pass-1 output| <= (8192 * 1151 + 53022 * 1023 + 1024) / 2048 = 31,095 (53,022: the
// largest AC row sum of |A|); every stream from 8-bit samples at a quantiser <= 255 is inside
// (|DC| <= 1024 + q/2, |AC| <= ~930 + q/2).  Strips outside go to the K2 fix-up launch.
// Checked against libjpeg's arithmetic on random and worst-case blocks of that domain
// (tools/idct_dot2_model.py).
#define RJ_DOT2_DC_MAX 1151
#define RJ_DOT2_AC_MAX 1023
// The VOP3P form v_dot2_i32_i16 with the constant pair in an SGPR and the accumulator as an
// operand (the builtin selects v_dot2c_i32_i16, whose accumulator is its destination: one extra
// v_mov per dot product that does not continue a chain -- 128 per block).
__device__ __forceinline__ int32_t dot2(uint32_t a, uint32_t k, int32_t c) {
  int32_t d;
  asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(k), "v"(c));
  return d;
}
__device__ __forceinline__ int32_t dot2z(uint32_t a, uint32_t k) {  // accumulator 0 (inline constant)
  int32_t d;
  asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(d) : "v"(a), "s"(k));
  return d;
}
#define RJ_PK(lo, hi) (uint32_t(uint16_t(int16_t(lo))) | (uint32_t(uint16_t(int16_t(hi))) << 16))
// byte offset of natural coefficient (row k, column c) in the pair layout
__host__ __device__ constexpr uint32_t rj_pair_slot(uint32_t k, uint32_t c) {
  return (c * 4u + ((k & 1u) ? 2u + (k >> 2) : (k >> 1) & 1u)) * 4u + ((k & 1u) ? (k >> 1) & 1u : k >> 2) * 2u;
}
// one pass over pairs p0 = (x0, x4), p1 = (x2, x6), p2 = (x1, x3), p3 = (x5, x7); ke0 / ke1:
// the (x0, x4) constants of the (x0 + x4) / (x0 - x4) terms, rnd added to both
__device__ __forceinline__ void islow_dot2_1d(uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3, uint32_t ke0,
                                              uint32_t ke1, int32_t rnd, int32_t t[8]) {
  const int32_t e0 = dot2(p0, ke0, rnd), e1 = dot2(p0, ke1, rnd);
  // the even butterfly folded into the accumulators: t10 / t13 = e0 +- tmp3, t11 / t12 = e1 +- tmp2
  // with tmp3 = (10703, 4433) . p1, tmp2 = (4433, -10704) . p1 (the negated pairs for the minus)
  const int32_t t10 = dot2(p1, RJ_PK(10703, 4433), e0), t13 = dot2(p1, RJ_PK(-10703, -4433), e0);
  const int32_t t11 = dot2(p1, RJ_PK(4433, -10704), e1), t12 = dot2(p1, RJ_PK(-4433, 10704), e1);
  const int32_t o0 = dot2(p3, RJ_PK(6437, 2260), dot2z(p2, RJ_PK(11363, 9633)));
  const int32_t o1 = dot2(p3, RJ_PK(-11362, -6436), dot2z(p2, RJ_PK(9633, -2259)));
  const int32_t o2 = dot2(p3, RJ_PK(2261, 9633), dot2z(p2, RJ_PK(6437, -11362)));
  const int32_t o3 = dot2(p3, RJ_PK(9633, -11363), dot2z(p2, RJ_PK(2260, -6436)));
  t[0] = t10 + o0;
  t[7] = t10 - o0;
  t[1] = t11 + o1;
  t[6] = t11 - o1;
  t[2] = t12 + o2;
  t[5] = t12 - o2;
  t[3] = t13 + o3;
  t[4] = t13 - o3;
}
// w: the block in the pair layout (scaled as above); o as idct_islow_block
__device__ __forceinline__ void idct_dot2_block(const uint32_t (&w)[32], uint32_t (&o)[16]) {
  uint32_t q[4][8];  // pass-2 pairs: q[j][r] = row r's pair j
  constexpr int kCa[4] = {0, 2, 1, 5}, kCb[4] = {4, 6, 3, 7};
#pragma unroll
  for (int j = 0; j < 4; j++) {
    int32_t ta[8], tb[8];
    const int ca = kCa[j], cb = kCb[j];
    islow_dot2_1d(w[4 * ca], w[4 * ca + 1], w[4 * ca + 2], w[4 * ca + 3], ca == 0 ? RJ_PK(16384, 8192) : RJ_PK(8192, 8192),
                  ca == 0 ? RJ_PK(16384, -8192) : RJ_PK(8192, -8192), 32768, ta);
    islow_dot2_1d(w[4 * cb], w[4 * cb + 1], w[4 * cb + 2], w[4 * cb + 3], RJ_PK(8192, 8192), RJ_PK(8192, -8192), 32768,
                  tb);
#pragma unroll
    for (int r = 0; r < 8; r++) q[j][r] = __builtin_amdgcn_perm(uint32_t(tb[r]), uint32_t(ta[r]), 0x07060302u);
  }
#pragma unroll
  for (int r = 0; r < 8; r++) {
    int32_t t[8];
    islow_dot2_1d(q[0][r], q[1][r], q[2][r], q[3][r], RJ_PK(8192, 8192), RJ_PK(8192, -8192), RJ_PASS2_RND, t);
    o[2 * r] = islow_pack4(islow_limit_biased(t[0]), islow_limit_biased(t[1]), islow_limit_biased(t[2]),
                           islow_limit_biased(t[3]));
    o[2 * r + 1] = islow_pack4(islow_limit_biased(t[4]), islow_limit_biased(t[5]), islow_limit_biased(t[6]),
                               islow_limit_biased(t[7]));
  }
}

// Exact ISLOW for coefficients outside the int32 domain above (only corrupt streams with large
// quantisers get here; K2 detects them per strip and records the row, which the K2 fix-up
// launch -- k_rows_fix, its own kernel, so none of this touches the common path's registers --
// decodes again with this arithmetic for the flagged strips):
// libjpeg jidctint.c as on LP64 (INT32/JLONG = long) with its RANGE_MASK wrap --
// oracle/jpeg_oracle.c idct_islow.  The output needs bits 18..27 of each pass-2 sum only, and
// pass 2 is linear with integer constants, so it is exact modulo 2^32 given the pass-1 outputs
// modulo 2^32: pass 1 runs in 64-bit (its outputs need bits 11..42 of the sums), pass 2 in
// wrapping 32-bit with full multiplies (v_mul_lo_u32; m24 would truncate).
// islow_1d in wrapping 32-bit arithmetic with full multiplies (pass 2 of the wide path).
__device__ __forceinline__ void islow_1d_wrap(const int32_t *xi, uint32_t rnd, int32_t t[8]) {
  const uint32_t x0 = xi[0], x1 = xi[1], x2 = xi[2], x3 = xi[3], x4 = xi[4], x5 = xi[5], x6 = xi[6], x7 = xi[7];
  uint32_t z1 = (x2 + x6) * uint32_t(RJ_FIX_0_541196100);
  const uint32_t tmp2 = z1 - x6 * uint32_t(RJ_FIX_1_847759065);
  const uint32_t tmp3 = z1 + x2 * uint32_t(RJ_FIX_0_765366865);
  const uint32_t e0 = ((x0 + x4) << 13) + rnd, e1 = ((x0 - x4) << 13) + rnd;
  const uint32_t t10 = e0 + tmp3, t13 = e0 - tmp3, t11 = e1 + tmp2, t12 = e1 - tmp2;
  uint32_t o0 = x7, o1 = x5, o2 = x3, o3 = x1;
  z1 = o0 + o3;
  uint32_t z2 = o1 + o2, z3 = o0 + o2, z4 = o1 + o3;
  const uint32_t z5 = (z3 + z4) * uint32_t(RJ_FIX_1_175875602);
  o0 *= uint32_t(RJ_FIX_0_298631336);
  o1 *= uint32_t(RJ_FIX_2_053119869);
  o2 *= uint32_t(RJ_FIX_3_072711026);
  o3 *= uint32_t(RJ_FIX_1_501321110);
  z1 *= uint32_t(-RJ_FIX_0_899976223);
  z2 *= uint32_t(-RJ_FIX_2_562915447);
  z3 = z3 * uint32_t(-RJ_FIX_1_961570560) + z5;
  z4 = z4 * uint32_t(-RJ_FIX_0_390180644) + z5;
  o0 += z1 + z3;
  o1 += z2 + z4;
  o2 += z2 + z3;
  o3 += z1 + z4;
  t[0] = int32_t(t10 + o3);
  t[7] = int32_t(t10 - o3);
  t[1] = int32_t(t11 + o2);
  t[6] = int32_t(t11 - o2);
  t[2] = int32_t(t12 + o1);
  t[5] = int32_t(t12 - o1);
  t[3] = int32_t(t13 + o0);
  t[4] = int32_t(t13 - o0);
}

// pass 1 of the wide path: 64-bit sums from the LDS block (zigzag coefficients, zigzag
// quantisers), outputs modulo 2^32 into v (natural order) -- all pass 2 needs.
__device__ __forceinline__ void idct_pass1_wide(const int16_t *zz, const uint16_t *qz, int32_t (&v)[64]) {
  constexpr uint8_t kZz[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
                               3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
                               10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
                               21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};
  auto X = [&](int nat) { return int64_t(zz[kZz[nat]]) * int64_t(qz[kZz[nat]]); };
#pragma unroll
  for (int c = 0; c < 8; c++) {
    int64_t z2 = X(16 + c), z3 = X(48 + c);
    int64_t z1 = (z2 + z3) * RJ_FIX_0_541196100;
    int64_t tmp2 = z1 - z3 * RJ_FIX_1_847759065;
    int64_t tmp3 = z1 + z2 * RJ_FIX_0_765366865;
    z2 = X(c);
    z3 = X(32 + c);
    int64_t tmp0 = (z2 + z3) * 8192, tmp1 = (z2 - z3) * 8192;
    const int64_t t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    tmp0 = X(56 + c);
    tmp1 = X(40 + c);
    tmp2 = X(24 + c);
    tmp3 = X(8 + c);
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int64_t z4 = tmp1 + tmp3;
    const int64_t z5 = (z3 + z4) * RJ_FIX_1_175875602;
    tmp0 *= RJ_FIX_0_298631336;
    tmp1 *= RJ_FIX_2_053119869;
    tmp2 *= RJ_FIX_3_072711026;
    tmp3 *= RJ_FIX_1_501321110;
    z1 *= -RJ_FIX_0_899976223;
    z2 *= -RJ_FIX_2_562915447;
    z3 = z3 * -RJ_FIX_1_961570560 + z5;
    z4 = z4 * -RJ_FIX_0_390180644 + z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    const int64_t rnd = 1 << 10;
    v[0 * 8 + c] = int32_t((t10 + tmp3 + rnd) >> 11);
    v[7 * 8 + c] = int32_t((t10 - tmp3 + rnd) >> 11);
    v[1 * 8 + c] = int32_t((t11 + tmp2 + rnd) >> 11);
    v[6 * 8 + c] = int32_t((t11 - tmp2 + rnd) >> 11);
    v[2 * 8 + c] = int32_t((t12 + tmp1 + rnd) >> 11);
    v[5 * 8 + c] = int32_t((t12 - tmp1 + rnd) >> 11);
    v[3 * 8 + c] = int32_t((t13 + tmp0 + rnd) >> 11);
    v[4 * 8 + c] = int32_t((t13 - tmp0 + rnd) >> 11);
  }
}

// pass 2 of the wide path (rows, wrapping 32-bit); output as idct_islow_block
__device__ __forceinline__ void idct_pass2_wrap(const int32_t (&v)[64], uint32_t (&o)[16]) {
#pragma unroll
  for (int r = 0; r < 8; r++) {
    int32_t t[8];
    islow_1d_wrap(v + r * 8, uint32_t(RJ_PASS2_RND), t);
    o[2 * r] = islow_pack4(islow_limit_biased(t[0]), islow_limit_biased(t[1]), islow_limit_biased(t[2]),
                           islow_limit_biased(t[3]));
    o[2 * r + 1] = islow_pack4(islow_limit_biased(t[4]), islow_limit_biased(t[5]), islow_limit_biased(t[6]),
                               islow_limit_biased(t[7]));
  }
}

// Colour conversion of the reference (src/rocjpeg_hip_kernels.cpp:1431-1443, same in every
// CSC kernel): BT.709-style constants, fmaf order as written there, u8 by v_cvt_pk_u8_f32.
__device__ __forceinline__ uint32_t cvt_u8(float f) { return __builtin_amdgcn_cvt_pk_u8_f32(f, 0, 0u) & 0xFFu; }

// R | G << 8 | B << 16, packed by v_cvt_pk_u8_f32 exactly as the reference's hipPack does.
__device__ __forceinline__ uint32_t csc_pixel_packed(uint32_t y, uint32_t u, uint32_t v) {
  const float fy = float(y), fu = float(u) - 128.0f, fv = float(v) - 128.0f;
  const float r = fmaf(1.5748f, fv, fy);
  const float g = fmaf(-0.4681f, fv, fmaf(-0.1873f, fu, fy));
  const float b = fmaf(1.8556f, fu, fy);
  return __builtin_amdgcn_cvt_pk_u8_f32(b, 2, __builtin_amdgcn_cvt_pk_u8_f32(g, 1, __builtin_amdgcn_cvt_pk_u8_f32(r, 0, 0u)));
}

__device__ __forceinline__ void csc_pixel(uint32_t y, uint32_t u, uint32_t v, uint8_t out[3]) {
  const uint32_t p = csc_pixel_packed(y, u, v);
  out[0] = uint8_t(p);
  out[1] = uint8_t(p >> 8);
  out[2] = uint8_t(p >> 16);
}

}  // namespace rj
